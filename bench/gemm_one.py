"""One GEMM shape, repeated: the target of rocprofv3 counter passes on a single kernel.

    CLOUD_AMD_GEMM_CORE=pp256 python bench/gemm_one.py 4096 4096 4096 --layout 0 --iters 50
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloud_amd.ops import raw  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("M", type=int)
    ap.add_argument("N", type=int)
    ap.add_argument("K", type=int)
    ap.add_argument("--layout", type=int, default=0, help="0 NT (forward), 1 NN (input grad)")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    torch.manual_seed(0)
    x = torch.randn(a.M, a.K, device="cuda").to(torch.bfloat16)
    if a.layout == 0:
        w = torch.randn(a.N, a.K, device="cuda").to(torch.bfloat16)
    else:
        w = torch.randn(a.K, a.N, device="cuda").to(torch.bfloat16)
    lay = raw.NT if a.layout == 0 else raw.NN
    for _ in range(3):
        raw.gemm(x, w, layout=lay)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        raw.gemm(x, w, layout=lay)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    print(f"{os.environ.get('CLOUD_AMD_GEMM_CORE', 'glds')} M={a.M} N={a.N} K={a.K} layout={a.layout}: "
          f"{ms * 1e3:.1f} us, {2.0 * a.M * a.N * a.K / ms / 1e9:.1f} TF/s")


if __name__ == "__main__":
    main()
