"""Step-level A/B of the data-parallel engine's knobs, run by the benches after their timed
region at N > 1.

The driver's multi-GPU scaling runs (``SCALE_rNN.json``) are the only multi-GPU evidence this
framework gets, so one such run must be able to settle the DP defaults that no single-GPU box
can measure: the per-bucket optimizer (``CLOUD_AMD_SLICED_OPT``), the bucket size
(``CLOUD_AMD_BUCKET_MB``) and the transport (``CLOUD_AMD_COMM``: ``torch.distributed`` over
RCCL vs the native communicator).  Each cell builds a fresh gradient reducer with its
settings, runs ``warmup`` untimed and ``steps`` (<= 5) timed training steps bracketed by a
device sync and a barrier (max over ranks), and reports ms/step and the exposed
communication; the reducer is then torn down (hooks removed, native communicator closed).
The headline ``value`` of the bench is untouched: this runs after it was measured.

Safety: a cell that raises is recorded with its error and the next cell runs; a cell that
does not finish within ``deadline_s`` (a hung collective) calls ``on_timeout`` from a
watchdog thread -- the benches print their result line with the cells measured so far and
exit, so the headline survives.
"""
from __future__ import annotations

import os
import threading
import time

DEFAULT_CELLS = [dict(transport=t, bucket_mb=b, sliced=s)
                 for t in ("torch", "rccl") for b in (16.0, 32.0, 64.0) for s in (False, True)]


def cells_from_env():
    """``CLOUD_AMD_BENCH_AB``: ``0`` off, ``1``/unset the default 12 cells, or a list
    ``transport:bucket_mb:sliced,...`` (e.g. ``torch:16:0,torch:16:1``)."""
    spec = os.environ.get("CLOUD_AMD_BENCH_AB", "1").strip()
    if spec in ("0", "off", "no", ""):
        return []
    if spec in ("1", "on", "yes"):
        return [dict(c) for c in DEFAULT_CELLS]
    out = []
    for item in spec.split(","):
        t, b, s = item.split(":")
        out.append(dict(transport=t, bucket_mb=float(b), sliced=s in ("1", "true", "on")))
    return out


class _Env:
    """Temporarily set environment variables."""

    def __init__(self, **kv):
        self.kv = {k: str(v) for k, v in kv.items()}
        self.old = {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.old[k] = os.environ.get(k)
            os.environ[k] = v
        return self

    def __exit__(self, *exc):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        return False


def teardown(reducer):
    """Remove a reducer's hooks and close its native communicator."""
    from ..parallel import ddp

    try:
        reducer.remove()
    finally:
        ddp._ACTIVE.discard(reducer)
        if getattr(reducer, "comm", None) is not None:
            reducer.comm.close()
            reducer.comm = None


def run_cells(build_reducer, set_reducer, train_step, optimizer, device, cells, steps=5, warmup=2,
              deadline_s=90.0, on_timeout=None, results=None):
    """Run every cell; returns (and fills ``results``, if given) one dict per cell.

    ``build_reducer(bucket_mb)`` -> a new GradAllReducer (built under the cell's environment);
    ``set_reducer(r)`` makes ``train_step()`` use it; ``optimizer`` is the fused optimizer
    (per-bucket update attached when the cell says ``sliced``)."""
    import torch

    from . import dist_env

    results = [] if results is None else results
    steps = max(1, min(int(steps), 5))
    cuda = device.type == "cuda"

    def sync():
        if cuda:
            torch.cuda.synchronize(device)

    state = {"cell": None, "t0": None, "done": False}

    def watchdog():
        while not state["done"]:
            time.sleep(1.0)
            t0 = state["t0"]
            if t0 is not None and time.time() - t0 > deadline_s and not state["done"]:
                results.append(dict(state["cell"], error="timeout after %.0f s (hung collective?)" % deadline_s))
                if on_timeout is not None:
                    on_timeout(results)
                os._exit(0)

    wd = threading.Thread(target=watchdog, name="dp-ab-watchdog", daemon=True)
    wd.start()
    try:
        for cell in cells:
            state["cell"], state["t0"] = dict(cell), time.time()
            red = None
            entry = dict(cell)
            try:
                with _Env(CLOUD_AMD_COMM=cell["transport"], CLOUD_AMD_SLICED_OPT="1" if cell["sliced"] else "0"):
                    red = build_reducer(cell["bucket_mb"])
                    entry["sliced_active"] = bool(red.attach_optimizer(optimizer)) if cell["sliced"] else False
                    entry["buckets"] = len(red.buckets)
                    entry["transport_active"] = red.describe()["transport"]
                set_reducer(red)
                for _ in range(warmup):
                    train_step()
                sync()
                dist_env.barrier()
                red.timing_start()
                sync()
                t0 = time.perf_counter()
                for _ in range(steps):
                    train_step()
                sync()
                dist_env.barrier()
                dt = dist_env.all_reduce_max(time.perf_counter() - t0, device)
                t = red.timing_summary()
                entry.update(ms_per_step=round(dt / steps * 1e3, 3),
                             exposed_comm_ms=round(dist_env.all_reduce_max(t["exposed_comm_ms"], device), 3),
                             allreduce_ms=round(dist_env.all_reduce_max(t["allreduce_ms"], device), 3),
                             steps=steps)
            except Exception as e:  # noqa: BLE001 - one cell's failure must not lose the others
                entry["error"] = "%s: %s" % (type(e).__name__, str(e)[:200])
            finally:
                if red is not None:
                    try:
                        red.optimizer = None
                        teardown(red)
                    except Exception as e:  # noqa: BLE001
                        entry.setdefault("error", "teardown: %s" % e)
            results.append(entry)
    finally:
        state["done"] = True
    return results


def best(results):
    """The fastest cell that ran (None if none did)."""
    ok = [r for r in results if "ms_per_step" in r]
    return min(ok, key=lambda r: r["ms_per_step"]) if ok else None
