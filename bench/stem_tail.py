#!/usr/bin/env python3
"""The ResNet-50 stem tail's three pooling kernels at the bench shape (z = [B, 112, 112, 64] bf16,
B = 1024 by default): BN + ReLU + 3x3/2 max-pool forward, the statistics-only max-pool backward
and the recomputing BN-backward apply (csrc/kernels/pool.hip).  Prints per-kernel microseconds
and the HBM bytes each must move at minimum (GB/s against that floor).  One JSON line."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloud_amd.ops import _ext  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    ext = _ext.load(required=True)
    st = _ext.stream_handle(torch.device("cuda"))
    N, H, W, C = a.batch, 112, 112, 64
    OH, OW = 56, 56
    torch.manual_seed(0)
    z = (torch.randn(N, H, W, C, device="cuda") * 2 + 0.3).to(torch.bfloat16)
    ss = torch.cat([torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.2])
    y = torch.empty(N, OH, OW, C, device="cuda", dtype=torch.bfloat16)
    idx = torch.empty(N, OH, OW, C, device="cuda", dtype=torch.uint8)
    dy = torch.randn(N, OH, OW, C, device="cuda").to(torch.bfloat16)
    parts = torch.empty(ext.maxpool_bnstats_parts(N, H, W, C), 2, C, device="cuda")
    coef = torch.randn(3 * C, device="cuda") * 0.01
    dz = torch.empty_like(z)
    zb, yb = z.numel() * 2, y.numel() * 2

    def fwd():
        ext.bn_relu_maxpool_s2k3(z.data_ptr(), ss.data_ptr(), y.data_ptr(), idx.data_ptr(), N, H, W, C, OH, OW, st)

    def stats():
        ext.maxpool_bwd_s2k3_bnstats(dy.data_ptr(), y.data_ptr(), idx.data_ptr(), z.data_ptr(), 0, parts.data_ptr(),
                                     N, H, W, C, OH, OW, st)

    def apply():
        ext.maxpool_bwd_s2k3_bnapply(dy.data_ptr(), y.data_ptr(), idx.data_ptr(), z.data_ptr(), coef.data_ptr(),
                                     dz.data_ptr(), N, H, W, C, OH, OW, st)

    fwd()
    row = {"batch": N}
    for name, fn, nbytes in (("fwd", fwd, zb + yb + yb // 2), ("bwd_stats", stats, zb + yb * 2 + yb // 2),
                             ("bwd_apply", apply, 2 * zb + yb * 2 + yb // 2)):
        us = timeit(fn)
        row[name + "_us"] = round(us, 1)
        row[name + "_floor_GBps"] = round(nbytes / us / 1e3, 1)
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
