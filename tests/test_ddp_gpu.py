"""Data parallelism through the hand-scheduled (fused) ResNet blocks on the GPU:
two ranks share the one GPU of the test box and talk over gloo (the 8-GPU run
uses RCCL; the DP engine is transport-agnostic).  Checks that every gradient
bucket is launched from the backward hooks / notify_grad_ready calls (before
finish()), and that replicas stay bit-identical."""
import os
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))



def _free_port():
    """An unused TCP port on 127.0.0.1 (bind to 0): fixed pid-based formulas collide across
    test cases and pytest-xdist workers."""
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]

def _worker(rank, world, port, out_dir, use_fused=True, emulate=1):
    """``emulate`` > 1 (with world 1): one process runs every replica's half-batch
    through forward/backward into the same arena (gradient accumulation) -- the
    single-process large-batch update the DP run must reproduce."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from cloud_amd.models import fused_block
    from cloud_amd.models.resnet import ResNet
    from cloud_amd.ops import softmax_cross_entropy
    from cloud_amd.optim import SGD
    from cloud_amd.parallel.ddp import GradAllReducer

    torch.cuda.set_device(0)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    m = ResNet((1, 1, 1, 1), num_classes=10, stem_channels_pad=5, device="cuda")
    for b in m.layers:
        b.fused_block = use_fused
    if rank == 1:
        with torch.no_grad():
            for p in m.parameters():
                p.add_(0.01)  # broadcast must undo this
    reps = world * emulate
    opt = SGD(m, learning_rate=0.05, momentum=0.9, grad_scale=1.0 / reps)
    red = GradAllReducer(opt.arenas, bucket_mb=0.05)
    red.broadcast_parameters()
    g = torch.Generator(device="cuda").manual_seed(1)
    X = torch.randn(8 * reps, 32, 32, 3, device="cuda", generator=g).to(torch.bfloat16)
    Y = torch.randint(0, 10, (8 * reps,), device="cuda", generator=g)
    xb, yb = X[rank * 8:(rank + 1) * 8].contiguous(), Y[rank * 8:(rank + 1) * 8].contiguous()
    fused = all(fused_block.can_fuse(b, torch.empty(1, 8, 8, b.conv1.cin, device="cuda", dtype=torch.bfloat16))
                for b in m.layers) and use_fused
    launched_in_backward, losses = [], []
    for _ in range(4):
        opt.zero_grad()
        if emulate > 1:
            for k in range(emulate):
                xk, yk = X[k * 8:(k + 1) * 8].contiguous(), Y[k * 8:(k + 1) * 8].contiguous()
                loss, _ = softmax_cross_entropy(m(xk), yk, denom=8)
                loss.backward()
            launched_in_backward.append(True)
        else:
            loss, _ = softmax_cross_entropy(m(xb), yb, denom=8)
            loss.backward()
            launched_in_backward.append(red._next == len(red.buckets))
        red.finish()
        opt.step()
        losses.append(float(loss))
    torch.save({"master": [a.master.detach().cpu() for a in opt.arenas], "fused": fused,
                "launched": launched_in_backward, "buckets": len(red.buckets), "losses": losses},
               os.path.join(out_dir, f"r{rank}.pt"))
    if world > 1:
        dist.destroy_process_group()


@pytest.mark.parametrize("use_fused", [True, False])
def test_ddp_two_ranks_through_fused_blocks(tmp_path, use_fused):
    world = 2
    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path), use_fused), nprocs=world, join=True)
    r = [torch.load(tmp_path / f"r{i}.pt", weights_only=True) for i in range(world)]
    assert r[0]["fused"] == use_fused and r[1]["fused"] == use_fused
    assert r[0]["buckets"] > 2
    assert all(r[0]["launched"]) and all(r[1]["launched"]), (r[0]["launched"], r[1]["launched"])
    for ai, (a, b) in enumerate(zip(r[0]["master"], r[1]["master"])):
        if not torch.equal(a, b):
            d = (a - b).abs()
            idx = torch.nonzero(d > 0).flatten()
            raise AssertionError("arena %d differs at %d/%d elems, max %.3g, first idx %s; losses %s %s"
                                 % (ai, idx.numel(), a.numel(), d.max().item(), idx[:8].tolist(),
                                    r[0]["losses"], r[1]["losses"]))
    assert all(torch.isfinite(torch.tensor(x["losses"])).all() for x in r)
    # ... and equal the single-process update over the full (2 x 8) batch, up to the
    # bf16 rounding of the gradient sums (accumulated in-arena vs summed on the wire)
    single = tmp_path / "single"
    single.mkdir()
    mp.spawn(_worker, args=(1, port + 3, str(single), use_fused, world), nprocs=1, join=True)
    ref = torch.load(single / "r0.pt", weights_only=True)
    # bf16 gradients round differently when two halves are summed on the wire vs
    # accumulated in the arena (1 ulp of |g| ~ 4 is 0.03): a handful of stem/first-layer
    # weights move by up to ~lr * 4 steps * 1 ulp, everything else agrees to 2e-3; the
    # fp32 BatchNorm parameters inherit those differences through 4 momentum steps
    # (measured: 1.0e-3 relative L2)
    for a, b in zip(r[0]["master"], ref["master"]):
        d = (a - b).abs()
        assert float(d.max()) < 2e-2, float(d.max())
        assert float((d > 2e-3).float().mean()) < 1e-3, int((d > 2e-3).sum())
        assert float(d.norm() / b.norm().clamp_min(1e-12)) < 5e-3
