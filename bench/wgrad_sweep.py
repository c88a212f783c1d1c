"""Weight-gradient micro-benchmark of the ResNet-50 layers with <= 64 output channels
(layer-1 3x3, the space-to-depth stem) and a layer-2 3x3 for contrast, at the bench's
per-GPU batch, over a range of split-K workgroup targets.

usage: python bench/wgrad_sweep.py [batch] [blocks,blocks,...]
One JSON line per (shape, target): time of conv_wgrad (split GEMM + reduce) and TF/s.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloud_amd.ops import raw  # noqa: E402

SHAPES = [  # H, Cin, Cout, k, stride, pad, tag
    (56, 64, 64, 3, 1, 1, "l1_c2"),
    (113, 16, 64, 4, 1, 1, "stem_s2d"),
    (28, 128, 128, 3, 1, 1, "l2_c2"),
]


def timeit(fn, iters=10, warm=3):
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


def check_fp32(H, cin, cout, k, s, p, nb=16):
    """relative L2 error of the bf16 weight gradient vs an fp32 torch reference"""
    x = torch.randn(nb, H, H, cin, device="cuda").to(torch.bfloat16)
    w = (torch.randn(cout, k, k, cin, device="cuda") * 0.05).to(torch.bfloat16)
    dy = torch.randn_like(raw.conv_fwd(x, w, s, p))
    gw = torch.zeros(w.shape, dtype=torch.float32, device="cuda")
    raw.conv_wgrad(dy, x, w.shape, s, p, out=gw, beta=0.0)
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (cout, cin, k, k),
                                      dy.float().permute(0, 3, 1, 2), stride=s, padding=p)
    ref = ref.permute(0, 2, 3, 1)
    return float((gw - ref).norm() / ref.norm())


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    targets = [int(t) for t in sys.argv[2].split(",")] if len(sys.argv) > 2 else [512, 1024, 2048]
    torch.manual_seed(0)
    for H, cin, cout, k, s, p, tag in SHAPES:
        e = check_fp32(H, cin, cout, k, s, p)
        print(json.dumps({"tag": tag, "fp32_rel_l2": e}), flush=True)
        assert e < 2e-2, e
        x = torch.randn(nb, H, H, cin, device="cuda").to(torch.bfloat16)
        w = (torch.randn(cout, k, k, cin, device="cuda") * 0.05).to(torch.bfloat16)
        dy = torch.randn_like(raw.conv_fwd(x, w, s, p))
        oh = dy.shape[1]
        fl = 2.0 * nb * oh * oh * cout * cin * k * k
        ref = None
        for t in targets:
            raw._WGRAD_BLOCKS = raw._WGRAD_BLOCKS_SMALLM = t
            gw = torch.zeros(w.shape, dtype=torch.float32, device="cuda")
            ms = timeit(lambda: raw.conv_wgrad(dy, x, w.shape, s, p, out=gw, beta=0.0))
            if ref is None:
                ref = gw.clone()
            err = float((gw - ref).norm() / ref.norm())
            print(json.dumps({"tag": tag, "blocks": t, "us": round(ms * 1000, 1),
                              "TF": round(fl / ms / 1e9, 1), "rel_vs_first": err}), flush=True)
        del x, dy


if __name__ == "__main__":
    main()
