"""HBM budgeting helpers (288 GB HBM3E per MI355X).

Used by the trial scheduler to pack several small trials onto one GPU and by
``describe()`` for job metadata.  Estimates are deliberately simple: bf16
weights + fp32 master + optimizer moments + grads per parameter, plus an
activation term measured from the first real step when available.
"""
from __future__ import annotations

import os

HBM_GB = float(os.environ.get("CLOUD_AMD_HBM_GB", 288))
_last = {"params": 0}


def param_bytes(n_params, optimizer="adam", compute_bytes=2):
    state = {"sgd": 4, "adam": 8, "adamw": 8, "rmsprop": 8}.get(optimizer, 8)
    return n_params * (compute_bytes + 4 + state + compute_bytes)


def note_model(model):
    try:
        _last["params"] = sum(p.numel() for p in model.parameters())
    except Exception:  # pragma: no cover
        pass
    return _last["params"]


def trials_per_gpu(trial_gb, hbm_gb=None, reserve=0.1, cap=64):
    """How many trials of ``trial_gb`` fit in one GPU's HBM, keeping ``reserve`` of it
    free.  ``cap`` is a sanity bound on processes per GPU, not a packing policy."""
    hbm_gb = HBM_GB if hbm_gb is None else hbm_gb
    if trial_gb <= 0:
        return cap
    return max(1, min(cap, int(hbm_gb * (1 - reserve) // trial_gb)))


def trial_footprint_gb(device=None):
    """Device memory a finished trial needed: the caching allocator's peak RESERVED
    bytes (what another process on the same GPU cannot use), in GiB; None on CPU."""
    try:
        import torch

        if torch.cuda.is_available() and torch.cuda.is_initialized():
            return torch.cuda.max_memory_reserved(device) / 2 ** 30
    except Exception:  # pragma: no cover
        pass
    return None


def array_gb(obj):
    """Bytes (GiB) of the arrays / tensors in ``obj`` (nested tuples, lists, dicts)."""
    if obj is None:
        return 0.0
    if isinstance(obj, (tuple, list)):
        return sum(array_gb(o) for o in obj)
    if isinstance(obj, dict):
        return sum(array_gb(o) for o in obj.values())
    n = getattr(obj, "nbytes", None)
    if n is None and hasattr(obj, "element_size") and hasattr(obj, "numel"):
        n = obj.element_size() * obj.numel()
    return float(n or 0) / 2 ** 30


def report_footprint(gb=None, path=None, extra_gb=0.0):
    """Write this worker's measured trial footprint for the scheduler
    (``CLOUD_AMD_FOOTPRINT_FILE``); returns the value written (None: nothing to report).
    ``extra_gb``: device memory the trial will still claim after the measurement (the
    validation arrays ``evaluate`` uploads at epoch end)."""
    path = path or os.environ.get("CLOUD_AMD_FOOTPRINT_FILE")
    gb = trial_footprint_gb() if gb is None else gb
    if not path or gb is None:
        return None
    gb = gb + float(extra_gb or 0.0)
    import json

    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        json.dump({"peak_gb": float(gb), "params": _last["params"]}, f)
    os.replace(tmp, path)
    return gb


def peak_allocated_gb(device=None):
    try:
        import torch

        if torch.cuda.is_available():
            return torch.cuda.max_memory_allocated(device) / 2 ** 30
    except Exception:  # pragma: no cover
        pass
    return 0.0
