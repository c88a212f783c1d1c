"""Error of the gradient all-reduce on the wire at 8 ranks: bf16
sums (the default for bf16 layers: half the xGMI bytes) against fp32 sums of the same
bf16 gradients (``reduce_dtype=fp32``), both measured against an exact fp64 sum.

8 gloo ranks on the CPU stand in for the 8 MI355X ranks: like RCCL's ring, gloo's
bf16 reduction rounds the running sum to bf16 after every addition."""
import json
import os
import sys

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD = 8
N = 1 << 16



def _free_port():
    """An unused TCP port on 127.0.0.1 (bind to 0): fixed pid-based formulas collide across
    test cases and pytest-xdist workers."""
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]

def _grads(rank):
    g = torch.Generator().manual_seed(100 + rank)
    # a shared signal plus per-rank noise (replica gradients are correlated), plus a few
    # large entries: the shape of real conv-weight gradients
    common = torch.randn(N, generator=torch.Generator().manual_seed(7))
    x = 0.5 * common + torch.randn(N, generator=g)
    x[:64] *= 50.0
    return x.to(torch.bfloat16)


def _worker(rank, port, out_dir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(WORLD), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    torch.set_num_threads(1)
    import torch.distributed as dist

    from cloud_amd.optim import SGD
    from cloud_amd.parallel.ddp import GradAllReducer

    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    res = {}
    for wire in ("bf16", "fp32"):
        p = torch.nn.Parameter(torch.zeros(N, dtype=torch.bfloat16))
        opt = SGD([p], learning_rate=0.0)
        red = GradAllReducer(opt.arenas, bucket_mb=0.03, reduce_dtype=wire)
        p.grad.copy_(_grads(rank))
        red.finish()
        res[wire] = p.grad.float().tolist()[:N]
    if rank == 0:
        with open(os.path.join(out_dir, "sums.json"), "w") as f:
            json.dump(res, f)
    dist.destroy_process_group()


def test_bf16_vs_fp32_wire_error_at_8_ranks(tmp_path):
    port = _free_port()
    mp.spawn(_worker, args=(port, str(tmp_path)), nprocs=WORLD, join=True)
    res = json.load(open(tmp_path / "sums.json"))
    exact = sum(_grads(r).double() for r in range(WORLD))
    err = {}
    for wire, vals in res.items():
        got = torch.tensor(vals, dtype=torch.float64)
        err[wire] = float((got - exact).norm() / exact.norm())
    ulp = 2.0 ** -8  # bf16 unit roundoff
    # fp32 on the wire: one rounding of the final sum back into the bf16 arena
    assert err["fp32"] < 0.6 * ulp, err
    # bf16 on the wire: up to WORLD-1 roundings of partial sums; bounded well below 1%
    assert err["bf16"] < 3.0 * ulp, err
    assert err["bf16"] >= err["fp32"]
    print("relative L2 error of the 8-rank gradient sum:", json.dumps(err))
