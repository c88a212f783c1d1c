"""A/B of the GEMM cores on the dense shapes of BERT-base (M = 8192 tokens) and
large ResNet 1x1 convolutions: TFLOP/s of the forward (NT), input-grad (NN)
and weight-grad (TN, split-K) kernels.  Run once per core:

    CLOUD_AMD_GEMM_CORE=glds python bench/gemm_core_ab.py
    CLOUD_AMD_GEMM_CORE=reg  python bench/gemm_core_ab.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloud_amd.ops import raw  # noqa: E402

SHAPES = [  # (M, N, K, tag)
    (8192, 2304, 768, "bert_qkv"), (8192, 768, 768, "bert_o"), (8192, 3072, 768, "bert_ffn1"),
    (8192, 768, 3072, "bert_ffn2"), (50176, 1024, 256, "rn_l3_c3"), (12544, 2048, 512, "rn_l4_c3"),
    (200704, 128, 512, "rn_l2_c1"), (4096, 4096, 4096, "square4k"), (8192, 8192, 8192, "square8k"),
]


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    os.environ.setdefault("CLOUD_AMD_GEMM_LIB", "never")  # the in-tree core, not the plain-GEMM library policy
    core = os.environ.get("CLOUD_AMD_GEMM_CORE", "default")
    torch.manual_seed(0)
    out = {"core": core, "shapes": []}
    for M, N, K, tag in SHAPES:
        a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        gw = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        r = {"tag": tag, "M": M, "N": N, "K": K}
        y = raw.gemm(a, w)
        ref = (a[:256].float() @ w.float().t())
        r["fwd_err"] = float((y[:256].float() - ref).norm() / ref.norm())
        yd = raw.gemm(dy, w, layout=raw.NN)
        refd = dy[:256].float() @ w.float()
        r["dgrad_err"] = float((yd[:256].float() - refd).norm() / refd.norm())
        raw.wgrad_into(dy, a, gw, beta=0.0)
        refw = dy.t().float() @ a.float()
        r["wgrad_err"] = float((gw.float() - refw).norm() / refw.norm())
        for name, fn in (("fwd", lambda: raw.gemm(a, w)), ("dgrad", lambda: raw.gemm(dy, w, layout=raw.NN)),
                         ("wgrad", lambda: raw.wgrad_into(dy, a, gw, beta=0.0)),
                         # the library comparator (hipBLASLt through torch.mm) on the same operands
                         ("blas_fwd", lambda: torch.mm(a, w.t())), ("blas_dgrad", lambda: torch.mm(dy, w)),
                         ("blas_wgrad", lambda: torch.mm(dy.t(), a))):
            ms = timeit(fn)
            r[name + "_ms"] = round(ms, 4)
            r[name + "_TF"] = round(fl / ms / 1e9, 1)
        print(json.dumps(r), flush=True)
        out["shapes"].append(r)
    print(json.dumps({"summary": core, "fwd_TF": [s["fwd_TF"] for s in out["shapes"]]}))


if __name__ == "__main__":
    main()
