#!/usr/bin/env python3
"""Cost of the dense-layer GEMM epilogues on BERT-base's FFN shapes (M = 8192): FFN1 forward
(NT 8192 x 3072 x 768) plain / + bias / + bias + GELU + kept pre-activation / + bias + ReLU +
pre-activation, and FFN2's input gradient (NN 8192 x 3072 x 768) plain / x GELU'(pre) /
x ReLU'(pre).  The GELU - ReLU difference is the activation arithmetic; ReLU - plain the extra
operand / output traffic.  One JSON line per case."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloud_amd.ops import raw  # noqa: E402


def timeit(fn, iters=30, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters * 1000.0, 1)


def main():
    M, N, K = 8192, 3072, 768
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    pre = torch.empty_like(y)
    fwd = {
        "plain": lambda: raw.gemm(x, w, out=y),
        "bias": lambda: raw.gemm(x, w, bias=b, out=y),
        "bias_gelu_pre": lambda: raw.gemm(x, w, bias=b, act="gelu", preact=pre, out=y),
        "bias_relu_pre": lambda: raw.gemm(x, w, bias=b, act="relu", preact=pre, out=y),
    }
    for k, f in fwd.items():
        print(json.dumps({"case": "ffn1_fwd_" + k, "us": timeit(f)}), flush=True)
    dy = torch.randn(M, K, device="cuda").to(torch.bfloat16)  # [M][K] x w [K][N] -> [M][N]
    w2 = (torch.randn(K, N, device="cuda") / K ** 0.5).to(torch.bfloat16)
    dx = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    bwd = {
        "plain": lambda: raw.gemm(dy, w2, layout=raw.NN, out=dx),
        "gelu_grad": lambda: raw.gemm(dy, w2, layout=raw.NN, dact_src=pre, act="gelu", out=dx),
        "relu_grad": lambda: raw.gemm(dy, w2, layout=raw.NN, dact_src=pre, act="relu", out=dx),
    }
    for k, f in bwd.items():
        print(json.dumps({"case": "ffn2_dgrad_" + k, "us": timeit(f)}), flush=True)


if __name__ == "__main__":
    main()
