#!/usr/bin/env python3
"""Memory-bound small-K GEMMs of ResNet-50 stages 1-2 (1x1 convs, NHWC) at batch
CLOUD_AMD_SMALLK_BATCH (default 1024): cloud_amd MFMA kernels (with and without the
BN-statistics epilogue -- the ResNet forward form, on the persistent resident-weight core
where it applies: compare runs with CLOUD_AMD_GEMM_PRW=0/1) vs hipBLASLt (torch.mm) vs a
plain copy of the output size.  Reports us and effective HBM TB/s (A read + C write).
One JSON line per case.  CLOUD_AMD_SMALLK_SET=conv3: the conv3 expansions of stages 2-4
(N = 512 / 1024 / 2048) -- compare CLOUD_AMD_GEMM_PRWN=0/1 (column-chunked persistent core)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench.gemm_shapes import timeit  # noqa: E402
from cloud_amd.ops import _ext, raw  # noqa: E402


def main():
    ext = _ext.load(required=True)
    dev = torch.device("cuda", 0)
    st = _ext.stream_handle(dev)
    B = int(os.environ.get("CLOUD_AMD_SMALLK_BATCH", "1024"))
    shapes = [(B * 56 * 56, 64, 256), (B * 56 * 56, 256, 64), (B * 56 * 56, 64, 64),
              (B * 56 * 56, 256, 128), (B * 28 * 28, 128, 512), (B * 28 * 28, 512, 128)]
    if os.environ.get("CLOUD_AMD_SMALLK_SET") == "conv3":
        shapes = [(B * 28 * 28, 128, 512), (B * 14 * 14, 256, 1024), (B * 7 * 7, 512, 2048)]
    for (M, K, N) in shapes:
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(N, K, device=dev).to(torch.bfloat16)
        c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        stats = raw.gemm_stats_buffer(M, N, K, dev)
        byts = (M * K + M * N) * 2

        def ours():
            ext.gemm_bf16(0, a.data_ptr(), K, w.data_ptr(), K, c.data_ptr(), N, M, N, K, 0, 0.0, st)

        def ours_st():
            ext.gemm_bf16(0, a.data_ptr(), K, w.data_ptr(), K, c.data_ptr(), N, M, N, K, stats.data_ptr(), 0.0, st)

        def blas():
            torch.mm(a, w.t(), out=c)

        src = torch.empty_like(c)

        def copy():
            c.copy_(src)

        def fill():
            c.fill_(1.0)

        def readsum():
            torch.sum(src, dtype=torch.float32)

        r = {"M": M, "K": K, "N": N, "stat_rows": stats.shape[0], "prw": os.environ.get("CLOUD_AMD_GEMM_PRW", "1"),
             "prwn": os.environ.get("CLOUD_AMD_GEMM_PRWN", "1")}
        for name, fn, b in [("ours", ours, byts), ("ours_stats", ours_st, byts), ("hipblaslt", blas, byts),
                            ("copy_C", copy, 2 * M * N * 2),
                            ("fill_C", fill, M * N * 2), ("read_C", readsum, M * N * 2)]:
            us = timeit(fn, iters=20, warm=3)
            r[name + "_us"] = round(us, 1)
            r[name + "_TBs"] = round(b / us / 1e6, 2)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
