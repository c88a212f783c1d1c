"""Process-group bootstrap for one-process-per-GPU jobs.

Reads the torchrun / cloud_amd-launcher environment (``RANK``, ``LOCAL_RANK``,
``WORLD_SIZE``, ``MASTER_ADDR``, ``MASTER_PORT``) and initialises
``torch.distributed`` with RCCL (backend ``"nccl"`` on ROCm) when a GPU is
present, gloo otherwise.  ``MASTER_ADDR`` defaults to 127.0.0.1 (container
hostnames may not resolve).
"""
from __future__ import annotations

import atexit
import datetime
import os

import torch
import torch.distributed as dist


def env_int(name, default):
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def rank():
    return env_int("RANK", 0)


def local_rank():
    return env_int("LOCAL_RANK", 0)


def world_size():
    return env_int("WORLD_SIZE", 1)


def init_distributed(backend=None, timeout_s=None, device=None):
    """Initialise the default process group if WORLD_SIZE > 1. Returns (rank, world, device)."""
    r, w, lr = rank(), world_size(), local_rank()
    if device is None:
        # CLOUD_AMD_SHARED_GPU=1 maps every local rank onto cuda:0: a rehearsal of the
        # multi-rank path on a one-GPU box (with CLOUD_AMD_DIST_BACKEND=gloo; RCCL
        # refuses two ranks on one device).
        from .. import config

        ordinal = 0 if config.get("CLOUD_AMD_SHARED_GPU") else lr
        device = torch.device("cuda", ordinal) if torch.cuda.is_available() else torch.device("cpu")
    if device.type == "cuda":
        torch.cuda.set_device(device)
    if w > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        backend = backend or os.environ.get("CLOUD_AMD_DIST_BACKEND") or (
            "nccl" if device.type == "cuda" else "gloo")
        if backend == "nccl":
            _rccl_defaults(w)
        timeout = datetime.timedelta(seconds=timeout_s or env_int("CLOUD_AMD_PG_TIMEOUT_S", 600))
        kw = {"device_id": device} if (backend == "nccl" and device.type == "cuda") else {}
        try:
            dist.init_process_group(backend, rank=r, world_size=w, timeout=timeout, **kw)
        except TypeError:
            dist.init_process_group(backend, rank=r, world_size=w, timeout=timeout)
        atexit.register(_shutdown)
    return r, w, device


def _rccl_defaults(world):
    """The launcher's xGMI RCCL defaults (``core.launcher.rccl_env``) for ranks started by
    another launcher (torchrun): the NCCL_* variables are read when the communicator is
    created, so setting them here (unless exported) still applies."""
    try:
        from ..core import launcher, topology

        for k, v in launcher.rccl_env(world, topology.xgmi_links_per_gpu(world)).items():
            if k.startswith("NCCL_"):
                os.environ.setdefault(k, v)
    except Exception:  # noqa: BLE001 - defaults only
        pass


def _shutdown():
    """Tear the default process group down before interpreter exit.  Left to the
    destructors, the store / gloo background threads can outlive their owners and
    the rank dies with ``terminate called without an active exception`` (SIGABRT)
    after its work is done -- seen as rare non-zero exit codes of finished jobs."""
    if dist.is_initialized():
        try:
            dist.destroy_process_group()
        except Exception:  # noqa: BLE001 - best effort at exit
            pass


def barrier():
    if dist.is_initialized():
        dist.barrier()


def all_reduce_max(x: float, device) -> float:
    if not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_gather_floats(x: float, device) -> list:
    """Every rank's value of ``x`` (rank order); ``[x]`` without a process group."""
    if not dist.is_initialized():
        return [x]
    t = torch.tensor([x], dtype=torch.float64, device=device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(o.item()) for o in out]


def allreduce_busbw(device, nbytes=64 << 20, iters=5, dtype=torch.float32):
    """One-shot all-reduce bus bandwidth in GB/s over the default group (nccl-tests
    convention: busbw = bytes * 2(n-1)/n / time; the slowest rank's time).  On an 8-GPU
    MI355X node this shows whether RCCL spreads a collective over the 7 xGMI links of a
    GPU (~150 GB/s per link) or rides one ring.  None without a multi-rank group."""
    if not dist.is_initialized() or dist.get_world_size() < 2:
        return None
    import time

    n = dist.get_world_size()
    t = torch.ones(max(nbytes // torch.tensor([], dtype=dtype).element_size(), 1), dtype=dtype, device=device)

    def sync():
        if t.is_cuda:
            torch.cuda.synchronize(t.device)

    dist.all_reduce(t)  # warm the communicator / channels
    sync()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        dist.all_reduce(t)
    sync()
    dt = all_reduce_max((time.perf_counter() - t0) / iters, device)
    size = t.numel() * t.element_size()
    return round(size * 2.0 * (n - 1) / n / dt / 1e9, 2)


def comm_probe(device, sizes_mb=(16, 64), iters=5, dtype=torch.bfloat16):
    """All-reduce bandwidth of BOTH data-plane transports on the same buffers: the
    ``torch.distributed`` process group (RCCL backend) and the native C++ communicator
    (``parallel/comm.RcclComm``, its own stream), bf16 at the gradient-bucket size and at
    64 MB.  One 8-GPU run then says which transport to make the default
    (``CLOUD_AMD_COMM``).  Per transport and size: ``busbw_gbs`` (nccl-tests convention,
    slowest rank) and ``algbw_gbs``; a transport that cannot run reports its error.
    Needs a multi-rank group (None otherwise); every rank must call it."""
    if not dist.is_initialized() or dist.get_world_size() < 2:
        return None
    import time

    n = dist.get_world_size()
    out = {}

    def timed(fn, t, sync_stream):
        fn(t)
        sync_stream()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn(t)
        sync_stream()
        dt = all_reduce_max((time.perf_counter() - t0) / iters, device)
        size = t.numel() * t.element_size()
        return {"busbw_gbs": round(size * 2.0 * (n - 1) / n / dt / 1e9, 2), "algbw_gbs": round(size / dt / 1e9, 2),
                "ms": round(dt * 1e3, 3)}

    def dev_sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    from ..parallel import comm as _comm

    out["bench_transport"] = _comm.backend()  # the data plane the timed steps used (CLOUD_AMD_COMM)
    bufs = {mb: torch.ones((mb << 20) // torch.tensor([], dtype=dtype).element_size(), dtype=dtype, device=device)
            for mb in sizes_mb}
    out["torch"] = {str(mb): timed(lambda t: dist.all_reduce(t), t, dev_sync) for mb, t in bufs.items()}
    if device.type == "cuda":
        try:
            from ..parallel.comm import RcclComm

            c = RcclComm(tag="comm_probe", device=device)
            try:
                out["rccl"] = {str(mb): timed(lambda t: c.all_reduce(t), t, c.synchronize) for mb, t in bufs.items()}
                out["rccl"]["init_s"] = round(all_reduce_max(c.init_seconds, device), 3)
            finally:
                c.close()
        except Exception as e:  # noqa: BLE001 - a probe reports, it never fails the bench
            out["rccl"] = {"error": "%s: %s" % (type(e).__name__, e)}
    return out
