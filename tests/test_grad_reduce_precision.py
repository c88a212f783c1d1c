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
    # BERT's fp32 arena (word-embedding table rows + LayerNorm / bias vectors): the
    # default bf16 wire reduces a bf16 copy and casts the sum back into the fp32 gradient
    bert = {}
    for wire in ("bf16", "fp32"):
        emb = torch.nn.Parameter(torch.zeros(EMB_ROWS, 768))
        ln = torch.nn.Parameter(torch.zeros(LN))
        opt = SGD([emb, ln], learning_rate=0.0)
        red = GradAllReducer(opt.arenas, bucket_mb=1.0, reduce_dtype=wire)
        ge, gl = _bert_grads(rank)
        emb.grad.copy_(ge)
        ln.grad.copy_(gl)
        red.finish()
        bert[wire] = {"emb": emb.grad.flatten().tolist(), "ln": ln.grad.tolist(),
                      "describe": red.describe()}
    # per-parameter wire (round 6): the embedding table alone on a bf16 wire, split into >= 4
    # pipelined chunks; the LayerNorm vectors keep fp32 sums
    os.environ["CLOUD_AMD_SPLIT_PARAM_MB"] = "0.5"
    emb = torch.nn.Parameter(torch.zeros(EMB_ROWS, 768))
    emb._ca_wire_dtype = torch.bfloat16
    ln = torch.nn.Parameter(torch.zeros(LN))
    opt = SGD([emb, ln], learning_rate=0.0)
    red = GradAllReducer(opt.arenas, bucket_mb=1.0)
    ge, gl = _bert_grads(rank)
    emb.grad.copy_(ge)
    ln.grad.copy_(gl)
    red.finish()
    bert["split"] = {"emb": emb.grad.flatten().tolist(), "ln": ln.grad.tolist(), "describe": red.describe()}
    if rank == 0:
        with open(os.path.join(out_dir, "sums.json"), "w") as f:
            json.dump(res, f)
        with open(os.path.join(out_dir, "bert.json"), "w") as f:
            json.dump(bert, f)
    dist.destroy_process_group()


EMB_ROWS, LN = 512, 9 * 768


def _bert_grads(rank):
    """Per-rank fp32 gradients shaped like BERT-base's fp32 arena: embedding rows that
    only some ranks touched (sparse token overlap: 1/4 of the rows per rank, scale ~1e-3)
    and dense LayerNorm gamma/beta gradients (scale ~1e-2)."""
    g = torch.Generator().manual_seed(500 + rank)
    emb = torch.randn(EMB_ROWS, 768, generator=g) * 1e-3
    emb[torch.rand(EMB_ROWS, generator=g) > 0.25] = 0.0
    ln = torch.randn(LN, generator=g) * 1e-2 + 0.02 * torch.randn(LN, generator=torch.Generator().manual_seed(3))
    return emb, ln


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

    bert = json.load(open(tmp_path / "bert.json"))
    emb_exact = sum(_bert_grads(r)[0].double() for r in range(WORLD)).flatten()
    ln_exact = sum(_bert_grads(r)[1].double() for r in range(WORLD))
    berr = {}
    for wire in ("bf16", "fp32"):
        for k, ex in (("emb", emb_exact), ("ln", ln_exact)):
            got = torch.tensor(bert[wire][k], dtype=torch.float64)
            berr[wire + "_" + k] = float((got - ex).norm() / ex.norm())
    # fp32 on the wire: fp32 sums (~1e-7); bf16 on the wire: a few bf16 roundings
    assert berr["fp32_emb"] < 1e-6 and berr["fp32_ln"] < 1e-6, berr
    assert berr["bf16_emb"] < 3.0 * ulp and berr["bf16_ln"] < 3.0 * ulp, berr
    d_bf, d_fp = bert["bf16"]["describe"], bert["fp32"]["describe"]
    assert d_bf["reduce_dtype"] == "bfloat16" and d_fp["reduce_dtype"] == "float32"
    assert d_bf["grad_dtypes"] == ["float32"]
    assert abs(d_bf["wire_mb_per_step"] * 2 - d_fp["wire_mb_per_step"]) < 0.05  # half the bytes
    for k, ex in (("emb", emb_exact), ("ln", ln_exact)):
        got = torch.tensor(bert["split"][k], dtype=torch.float64)
        berr["split_" + k] = float((got - ex).norm() / ex.norm())
    assert berr["split_emb"] < 3.0 * ulp and berr["split_ln"] < 1e-6, berr
    d_sp = bert["split"]["describe"]
    assert d_sp["split_params"] and d_sp["split_params"][0]["chunks"] >= 4
    assert d_sp["split_params"][0]["wire"] == "bfloat16"
    assert d_bf["wire_mb_per_step"] - 0.05 < d_sp["wire_mb_per_step"] < d_fp["wire_mb_per_step"]
    print("BERT fp32-arena 8-rank sums, relative L2 error:", json.dumps(berr))
