"""The RCCL data plane of the 8-GPU run, executed on the one-GPU box.

A world-1 ``nccl`` (RCCL) process group plus a :class:`GradAllReducer` forced to
``world=2`` takes exactly the branches a multi-GPU run takes -- hooks launch buckets
during backward, the comm side stream, ``work.wait()`` on it, the wire-dtype copy back,
the per-bucket timing events -- for both transports:

* ``torch``: ``torch.distributed.all_reduce`` on the side stream (``parallel/ddp.py``
  ``_launch``, ``_device_timed`` branch);
* ``rccl``: the native C++ communicator (``csrc/comm/rccl_comm.cpp``) on its own stream,
  joined before the optimizer.

An all-reduce over one rank is the identity, so with ``grad_scale`` = 1 the master
weights must be BITWISE those of the same steps without DP (ResNet kernels are
deterministic), for bf16 and fp32 wires.  The step must add no host synchronisation
(``torch.cuda.set_sync_debug_mode`` counts every synchronising call), and the timing
summary must be finite with the exposed communication inside the step.

What each wire case can and cannot see: with the bf16 wire the bf16 arenas are reduced IN
PLACE, and an in-place all-reduce over one rank is a no-op -- a collective ordered too early
against its producers would still leave the right bytes.  Only the fp32-wire case checks
producer -> collective -> consumer ordering for the bf16 arenas, because their gradients go
through the comm stream's copy into the fp32 wire buffer and back: a copy that ran before the
producing kernels (or a copy back after the optimizer read) changes the bits.  The fp32-wire
case is therefore mandatory for both transports; the bf16 case covers the fp32 arenas'
bf16 round trip and the launch / timing branches.

Reference: the MirroredStrategy / MWMS gradient all-reduce the reference relies on,
``/root/reference/src/python/tensorflow_cloud/core/preprocess.py:137-146`` and
``core/tests/testdata/mnist_example_using_ctl.py:129,155-157``.
"""
import math
import os
import sys
import warnings

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _count_syncs(fn):
    """Number of synchronising CUDA/HIP calls ``fn`` makes (sync debug mode 'warn')."""
    torch.cuda.synchronize()
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        torch.cuda.set_sync_debug_mode("warn")
        try:
            fn()
        finally:
            torch.cuda.set_sync_debug_mode("default")
    return sum("synchroniz" in str(x.message).lower() for x in w)


def _worker(rank, port, out_path, transport, wire, sliced=False):
    os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      CLOUD_AMD_COMM=transport, CLOUD_AMD_GRAD_REDUCE_DTYPE=wire,
                      CLOUD_AMD_SLICED_OPT="1" if sliced else "0")  # opt-in since round 6
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from cloud_amd.models.resnet import ResNet
    from cloud_amd.ops import softmax_cross_entropy
    from cloud_amd.optim import SGD
    from cloud_amd.parallel.ddp import GradAllReducer

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    g = torch.Generator(device="cuda").manual_seed(1)
    X = torch.randn(4, 16, 32, 32, 3, device="cuda", generator=g).to(torch.bfloat16)
    Y = torch.randint(0, 10, (4, 16), device="cuda", generator=g)

    def build():
        torch.manual_seed(0)
        m = ResNet((1, 1, 1, 1), num_classes=10, stem_channels_pad=5, device="cuda")
        return m, SGD(m, learning_rate=0.05, momentum=0.9, grad_scale=1.0)

    def step(m, opt, red, i):
        opt.zero_grad()
        loss, _ = softmax_cross_entropy(m(X[i]), Y[i], denom=16)
        loss.backward()
        if red is not None:
            red.finish()
        elif wire == "bf16":
            # the bf16 wire rounds fp32 arenas' gradients (BatchNorm) to bf16 and back:
            # the reference applies the same rounding so the comparison stays bitwise
            for a in opt.arenas:
                if a.grad.dtype == torch.float32:
                    a.grad.copy_(a.grad.to(torch.bfloat16))
        opt.step()
        return loss

    # reference: the same steps with no data parallelism
    m0, o0 = build()
    for i in range(4):
        step(m0, o0, None, i)
    torch.cuda.synchronize()
    ref = [a.master.detach().cpu().clone() for a in o0.arenas]
    syncs_ref = _count_syncs(lambda: step(m0, o0, None, 0))

    m1, o1 = build()
    red = GradAllReducer(o1.arenas, bucket_mb=0.05, world=2)  # forced multi-rank reducer
    info = {"describe": red.describe(), "side": red._side is not None, "native": red.comm is not None,
            "device_timed": red._device_timed, "buckets": len(red.buckets)}
    red.broadcast_parameters()  # C2 over the same transport (one rank: identity)
    info["sliced"] = red.attach_optimizer(o1) if sliced else False
    red.probe_readiness()
    launched = []
    step(m1, o1, red, 0)  # first collective: communicator setup outside the timed steps
    red.timing_start()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for i in range(1, 4):
        opt = o1
        opt.zero_grad()
        loss, _ = softmax_cross_entropy(m1(X[i]), Y[i], denom=16)
        loss.backward()
        launched.append(red._next)  # buckets launched by the hooks during backward
        red.finish()
        opt.step()
    t1.record()
    torch.cuda.synchronize()
    ms_per_step = t0.elapsed_time(t1) / 3
    summary = red.timing_summary()
    info["budget"] = red.overlap_budget()
    got = [a.master.detach().cpu().clone() for a in o1.arenas]
    syncs_dp = _count_syncs(lambda: step(m1, o1, red, 0))
    if red.comm is not None:
        red.comm.close()
    dist.destroy_process_group()
    torch.save({"ref": ref, "got": got, "info": info, "summary": summary, "ms_per_step": ms_per_step,
                "launched": launched, "syncs_ref": syncs_ref, "syncs_dp": syncs_dp}, out_path)


@pytest.mark.parametrize("transport", ["torch", "rccl"])
@pytest.mark.parametrize("wire,sliced", [("bf16", True), ("fp32", True), ("fp32", False)])
def test_rccl_data_plane_world1_forced_multirank(tmp_path, transport, wire, sliced):
    """``sliced``: the fused SGD runs per bucket on its own stream as each bucket's collective
    completes (``attach_optimizer``, opt-in ``CLOUD_AMD_SLICED_OPT=1``); the weights must still be BITWISE
    those of the whole-arena step without DP."""
    out = str(tmp_path / "r.pt")
    mp.spawn(_worker, args=(_free_port(), out, transport, wire, sliced), nprocs=1, join=True)
    r = torch.load(out, weights_only=True)
    info = r["info"]
    assert info["device_timed"] is True
    assert info["sliced"] is sliced
    b = info["budget"]  # overlap budget: per-bucket readiness before the end of backward
    assert b is not None and b["steps"] == 4 and len(b["buckets"]) == info["buckets"]
    assert any(x["ready_before_bwd_end_ms"] > 0 for x in b["buckets"])
    assert all(math.isfinite(v) and v >= 0 for v in b["predicted_exposed_comm_ms"].values())
    if transport == "rccl":
        assert info["native"] and info["describe"]["transport"] == "native RcclComm"
    else:
        assert info["side"] and info["describe"]["transport"] == "torch.distributed(nccl)"
    assert info["describe"]["reduce_dtype"] == {"bf16": "bfloat16", "fp32": "float32"}[wire]
    assert info["buckets"] > 2
    # every bucket but the tail ones launched from backward hooks, before finish()
    assert all(n >= 1 for n in r["launched"]), r["launched"]
    # all-reduce over one rank is the identity: bitwise the no-DP update
    for a, b in zip(r["got"], r["ref"]):
        assert torch.equal(a, b), float((a - b).abs().max())
    s = r["summary"]
    assert s["timing"] == "device_events" and s["steps"] == 3
    assert math.isfinite(s["allreduce_ms"]) and math.isfinite(s["exposed_comm_ms"])
    assert s["allreduce_ms"] > 0.0
    assert 0.0 <= s["exposed_comm_ms"] <= r["ms_per_step"], (s, r["ms_per_step"])
    # no host synchronisation added by the data plane (the reference's one-off first-use sync
    # of a kernel library may show up on its side only)
    assert r["syncs_dp"] <= r["syncs_ref"], (r["syncs_dp"], r["syncs_ref"])
