"""Loader for the in-tree gfx950 extension (``cloud_amd/_C*.so``).

Policy (fail loudly, never silently fall back on a GPU):

* ``CLOUD_AMD_OPS=native`` (default): CUDA(HIP) tensors go through the HIP
  kernels; if the extension cannot be loaded while a GPU is present, ops raise.
* ``CLOUD_AMD_OPS=torch``: stock PyTorch implementations everywhere (used by
  the stock comparator in ``bench/`` and by CPU unit tests).

CPU tensors always use the PyTorch reference path (the kernels are gfx950-only).
"""
from __future__ import annotations

import importlib
import os
import threading

import torch

_lock = threading.Lock()
_ext = None
_err = None


_OPS_MODE = []


def ops_mode() -> str:
    """``CLOUD_AMD_OPS`` (read once per process: asked on every op)."""
    if not _OPS_MODE:
        _OPS_MODE.append(os.environ.get("CLOUD_AMD_OPS", "native").lower())
    return _OPS_MODE[0]


def load(required: bool = False):
    """Return the ``cloud_amd._C`` module (or None when unavailable and not required)."""
    global _ext, _err
    if _ext is not None:
        return _ext
    with _lock:
        if _ext is None and _err is None:
            try:
                _ext = importlib.import_module("cloud_amd._C")
            except Exception as e:  # pragma: no cover - depends on build state
                _err = e
    if _ext is None and required:
        raise RuntimeError(
            "cloud_amd native extension is not built/loadable (run `python -m cloud_amd._build`): "
            f"{_err!r}")
    return _ext


def use_native(*tensors) -> bool:
    """True when the HIP path must be used for these tensors."""
    if ops_mode() == "torch":
        return False
    if not tensors or not all(isinstance(t, torch.Tensor) and t.is_cuda for t in tensors if t is not None):
        return False
    load(required=True)
    return True


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_handle(device=None) -> int:
    """The current HIP stream of ``device`` as an integer handle.  Called once per kernel
    launch: the raw-stream query costs ~0.3 us where ``torch.cuda.current_stream(d).cuda_stream``
    (a Stream object per call) cost ~4.3 us of host time (BERT step: ~300 launches,
    profiles/r6_s12)."""
    if _RAW_STREAM is not None:
        if isinstance(device, torch.device) and device.index is not None:
            return _RAW_STREAM(device.index)
        if isinstance(device, int):
            return _RAW_STREAM(device)
        if device is None or (isinstance(device, torch.device) and device.type == "cuda"):
            return _RAW_STREAM(torch.cuda.current_device())
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()
