#!/usr/bin/env python3
"""BERT-base's N = 768 GEMMs at M = 8192 (FFN2 forward, QKV / FFN1 input gradients, attention
output): the in-tree dispatch (128 x 64 tiles, 768 tiles = 3 rounds) against split-K into fp32
slabs on 128 x 128 tiles (+ the streaming reduce), and hipBLASLt (torch.mm) in the same
process.  One JSON line per (shape, layout)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloud_amd.ops import _ext, raw  # noqa: E402


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
    return s.elapsed_time(e) / iters * 1000.0


def main():
    ext = _ext.load(required=True)
    st = _ext.stream_handle(torch.device("cuda"))
    M = 8192
    for N, K, layout in [(768, 3072, raw.NT), (768, 768, raw.NT), (768, 2304, raw.NN), (768, 3072, raw.NN),
                         (768, 768, raw.NN)]:
        torch.manual_seed(0)
        a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") if layout == raw.NT else torch.randn(K, N, device="cuda")).to(torch.bfloat16)
        wl = w.t() if layout == raw.NT else w
        ref = a.float() @ wl.float()
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        row = {"M": M, "N": N, "K": K, "layout": "NT" if layout == raw.NT else "NN"}
        row["ours_us"] = round(timeit(lambda: raw.gemm(a, w, out=out, layout=layout)), 1)
        for splits in (2, 3, 4):
            ws = torch.empty(splits * M * N, device="cuda", dtype=torch.float32)

            def f():
                ext.gemm_splitk(layout, a.data_ptr(), K, w.data_ptr(), w.stride(0), out.data_ptr(), 1, 0.0, M, N, K,
                                splits, ws.data_ptr(), st)

            row["splitk%d_us" % splits] = round(timeit(f), 1)
            row["splitk%d_rel" % splits] = float((out.float() - ref).norm() / ref.norm())
        row["hipblaslt_us"] = round(timeit(lambda: torch.mm(a, wl)), 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
