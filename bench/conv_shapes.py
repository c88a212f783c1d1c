"""Micro-benchmark of the implicit-GEMM conv kernels on ResNet-50 (batch 256)
3x3 / strided shapes: fwd, dgrad, wgrad time and TFLOP/s per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloud_amd.ops import raw  # noqa: E402

SHAPES = [  # N, H, Cin, Cout, k, stride, pad, tag
    (256, 56, 64, 64, 3, 1, 1, "l1_c2"), (256, 28, 128, 128, 3, 1, 1, "l2_c2"),
    (256, 56, 128, 128, 3, 2, 1, "l2_c2_s2"), (256, 14, 256, 256, 3, 1, 1, "l3_c2"),
    (256, 7, 512, 512, 3, 1, 1, "l4_c2"), (256, 56, 256, 512, 1, 2, 0, "l2_ds"),
    (256, 224, 8, 64, 7, 2, 3, "stem"),
]


def timeit(fn, iters=10, warm=2):
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
    only = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] != "all" else None
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else None  # override the per-shape batch
    for N, H, Cin, Cout, k, s, p, tag in SHAPES:
        N = batch or N
        if only and tag != only:
            continue
        x = torch.randn(N, H, H, Cin, device="cuda").to(torch.bfloat16)
        w = (torch.randn(Cout, k, k, Cin, device="cuda") * 0.05).to(torch.bfloat16)
        y = raw.conv_fwd(x, w, s, p)
        dy = torch.randn_like(y)
        gw = torch.zeros_like(w)
        OH = y.shape[1]
        fl = 2.0 * N * OH * OH * Cout * Cin * k * k
        r = {"tag": tag}
        for name, fn in (("fwd", lambda: raw.conv_fwd(x, w, s, p)),
                         ("dgrad", lambda: raw.conv_dgrad(dy, w, x.shape, s, p)),
                         ("wgrad", lambda: raw.conv_wgrad(dy, x, w.shape, s, p, out=gw, beta=0.0))):
            ms = timeit(fn)
            r[name + "_us"] = round(ms * 1000, 1)
            r[name + "_TF"] = round(fl / ms / 1e9, 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
