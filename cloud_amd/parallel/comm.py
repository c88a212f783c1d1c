"""Python face of the native RCCL communicator (``csrc/comm/rccl_comm.cpp``).

``RcclComm`` bootstraps one ``ncclComm_t`` per process: rank 0 creates the
128-byte unique id and publishes it through the rendezvous store of the default
``torch.distributed`` process group (TCPStore at MASTER_ADDR:MASTER_PORT); all
ranks then join with ``ncclCommInitRank``.  Collectives run on the
communicator's own high-priority HIP stream, ordered after the compute stream
by an event, so the DP engine (:mod:`cloud_amd.parallel.ddp`) can overlap
bucket all-reduces with the rest of backward and ``join`` the compute stream
only before the optimizer step.

Robustness: the bootstrap has a deadline (``CLOUD_AMD_COMM_INIT_TIMEOUT_S``, default 300 s):
a non-root rank waits for the unique id with ``store.wait(..., timeout)``, and the C++
init runs ``ncclCommInitRankConfig`` non-blocking, polled until every peer joined or the
deadline passed -- then the half-built communicator is aborted and ``TimeoutError`` is
raised, so a peer that HANGS before joining fails the job promptly instead of stalling
every rank until the launcher's timeout.  ``init_seconds`` records how long the init took.

Selection: ``CLOUD_AMD_COMM=rccl`` (native communicator) or ``torch`` (default:
``torch.distributed`` with the RCCL backend).  The native path is opt-in until
it has been validated on a multi-GPU node; both run RCCL underneath.
"""
from __future__ import annotations

import importlib
import itertools
import os

import torch
import torch.distributed as dist

_DTYPES = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int32: 3, torch.int64: 4, torch.uint8: 5}
_OPS = {"sum": 0, "max": 1, "min": 2, "avg": 3}
_ctr = itertools.count()


def backend() -> str:
    return os.environ.get("CLOUD_AMD_COMM", "torch").lower()


def load():
    return importlib.import_module("cloud_amd._comm")


def _stream(device=None):
    return torch.cuda.current_stream(device).cuda_stream


def init_timeout_s() -> float:
    return float(os.environ.get("CLOUD_AMD_COMM_INIT_TIMEOUT_S", "300"))


def exchange_unique_id(store, key, rank, make_uid, timeout_s):
    """Rank 0 publishes ``make_uid()`` under ``key``; every other rank waits for it at most
    ``timeout_s`` seconds (``TimeoutError`` naming the key otherwise -- rank 0 hung or died
    before publishing).  ``store`` is any c10d-style store (``set`` / ``get`` / ``wait``)."""
    import datetime

    if rank == 0:
        uid = make_uid()
        store.set(key, uid)
        return bytes(uid)
    try:
        store.wait([key], datetime.timedelta(seconds=timeout_s))
    except Exception as e:  # c10d raises RuntimeError / DistStoreError on its deadline
        raise TimeoutError("rank %d: RCCL unique id %r not published by rank 0 within %.1f s (%s)"
                           % (rank, key, timeout_s, e)) from e
    return bytes(store.get(key))


class RcclComm:
    def __init__(self, rank=None, world=None, device=None, store=None, tag=None, timeout_s=None):
        ext = load()
        self.rank = dist.get_rank() if rank is None else rank
        self.world = dist.get_world_size() if world is None else world
        dev = torch.device("cuda") if device is None else torch.device(device)
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.timeout_s = init_timeout_s() if timeout_s is None else float(timeout_s)
        key = "cloud_amd/rccl_uid/%s" % (tag if tag is not None else next(_ctr))
        if self.world > 1 and store is not False:
            store = store or dist.distributed_c10d._get_default_store()
            uid = exchange_unique_id(store, key, self.rank, ext.unique_id, self.timeout_s)
        else:
            uid = ext.unique_id()
        self.c = ext.Comm(self.world, self.rank, bytes(uid), self.device.index, self.timeout_s)
        self.init_seconds = float(self.c.init_seconds)

    def _args(self, t):
        assert t.is_cuda and t.is_contiguous(), "collectives need contiguous device tensors"
        return t.data_ptr(), t.numel(), _DTYPES[t.dtype]

    def all_reduce(self, t, op="sum"):
        p, n, d = self._args(t)
        self.c.all_reduce(p, n, d, _OPS[op], _stream(t.device))

    def broadcast(self, t, root=0):
        p, n, d = self._args(t)
        self.c.broadcast(p, n, d, root, _stream(t.device))

    def reduce_scatter(self, out, inp, op="sum"):
        self.c.reduce_scatter(inp.data_ptr(), out.data_ptr(), out.numel(), _DTYPES[out.dtype], _OPS[op],
                              _stream(out.device))

    def all_gather(self, out, inp):
        self.c.all_gather(inp.data_ptr(), out.data_ptr(), inp.numel(), _DTYPES[inp.dtype], _stream(inp.device))

    def join(self, device=None):
        """The current (compute) stream waits for every collective issued so far."""
        self.c.join(_stream(device or self.device))

    def synchronize(self):
        self.c.synchronize()

    def healthy(self) -> bool:
        return self.c.async_error() == 0

    def abort(self):
        self.c.abort()

    def start_watchdog(self, interval_s=1.0, on_error=None):
        """Background thread polling ncclCommGetAsyncError: on an
        asynchronous RCCL failure the communicator is aborted (unblocking any rank stuck
        in a collective) and ``on_error(code)`` runs (default: log + os._exit(75) so the
        launcher's watchdog tears the job down)."""
        import threading

        def loop():
            while not self._stop.wait(interval_s):
                try:
                    err = self.c.async_error()
                except RuntimeError:
                    return
                if err not in (0, 7):  # 7 = ncclInProgress
                    self.c.abort()
                    if on_error is not None:
                        on_error(err)
                    else:
                        import sys

                        print("[cloud_amd] RCCL async error %d: communicator aborted" % err, file=sys.stderr,
                              flush=True)
                        os._exit(75)
                    return

        self._stop = threading.Event()
        self._wd = threading.Thread(target=loop, name="rccl-watchdog", daemon=True)
        self._wd.start()
        return self._wd

    def stop_watchdog(self):
        if getattr(self, "_stop", None) is not None:
            self._stop.set()

    def close(self):
        self.stop_watchdog()
        self.c.destroy()
