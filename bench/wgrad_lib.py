#!/usr/bin/env python3
"""Dense weight gradient out[N_out, K_in] (+)= dy[M, N_out]^T x[M, K_in] with fp32 out, the
BERT-base shapes (M = 64 x 128 tokens): the in-tree split-K kernel + fixed-order slab
reduce (raw.wgrad_into) against hipBLASLt's bf16 -> fp32 GEMM (torch mm / addmm with
out_dtype).  Prints one line per shape: microseconds per call and max error vs fp32."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(fn, iters=30):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    from cloud_amd.ops import _ext, raw

    _ext.load(required=True)
    M = int(os.environ.get("WGRAD_M", "8192"))
    for n, k in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        torch.manual_seed(n + k)
        dy = torch.randn(M, n, device="cuda").to(torch.bfloat16)
        x = torch.randn(M, k, device="cuda").to(torch.bfloat16)
        ref = dy.float().t() @ x.float()
        out = torch.zeros(n, k, device="cuda")
        raw.wgrad_into(dy, x, out, beta=0.0)
        e_ours = (out - ref).abs().max().item()
        t_ours = _time(lambda: raw.wgrad_into(dy, x, out, beta=1.0))
        row = f"n={n} k={k} M={M} ours {t_ours:7.1f} us err {e_ours:.3g}"
        try:
            o2 = torch.mm(dy.t(), x, out_dtype=torch.float32)
            e_mm = (o2 - ref).abs().max().item()
            t_mm = _time(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
            row += f" | lib mm {t_mm:7.1f} us err {e_mm:.3g}"
        except Exception as ex:  # noqa: BLE001
            row += f" | lib mm n/a ({type(ex).__name__}: {str(ex)[:80]})"
        try:
            o3 = torch.zeros(n, k, device="cuda")
            torch.addmm(o3, dy.t(), x, out_dtype=torch.float32, out=o3)
            e_am = (o3 - ref).abs().max().item()
            t_am = _time(lambda: torch.addmm(o3, dy.t(), x, out_dtype=torch.float32, out=o3))
            row += f" | lib addmm(out=C) {t_am:7.1f} us err {e_am:.3g}"
        except Exception as ex:  # noqa: BLE001
            row += f" | lib addmm n/a ({type(ex).__name__}: {str(ex)[:80]})"
        print(row, flush=True)


if __name__ == "__main__":
    main()
