"""Time the fused 1x1 input+weight gradient (``raw.conv1x1_dgrad_wgrad_bnbwd``) on ResNet-50's
stage-1 shape (conv3: K = 256 -> N = 64, M = batch x 56 x 56), with and without the
BN-statistics epilogue.  The kernel form comes from the environment (``CLOUD_AMD_XA_DW_DEPTH``
is read once per process), so A/B runs are separate processes.

    python bench/xa_dw_bench.py --batch 1024 --iters 20
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from cloud_amd.ops import raw  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--hw", type=int, default=56)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    N, H, W, K, C = a.batch, a.hw, a.hw, 256, 64
    M = N * H * W
    dy = torch.randn((N, H, W, K), device=dev, generator=g).to(torch.bfloat16)
    z = torch.randn((N, H, W, K), device=dev, generator=g).to(torch.bfloat16)
    mask = torch.randint(0, 256, (M, K // 8), device=dev, generator=g, dtype=torch.int32).to(torch.uint8)
    coef = torch.randn(3 * K, device=dev, generator=g) * 0.1
    w = (torch.randn((K, 1, 1, C), device=dev, generator=g) * 0.05).to(torch.bfloat16)
    y = torch.randn((N, H, W, C), device=dev, generator=g).to(torch.bfloat16)
    z2 = torch.randn((N, H, W, C), device=dev, generator=g).to(torch.bfloat16)
    m2 = torch.randint(0, 256, (M, C // 8), device=dev, generator=g, dtype=torch.int32).to(torch.uint8)
    out = {"depth": os.environ.get("CLOUD_AMD_XA_DW_DEPTH", "default"), "M": M}
    for name, bn in (("bn", (z2, m2)), ("plain", None)):
        dw = torch.zeros((K, 1, 1, C), device=dev, dtype=torch.float32)
        for _ in range(3):
            dw.zero_()
            r = raw.conv1x1_dgrad_wgrad_bnbwd(dy, z, mask, coef, w, y, dw, bn=bn, dw_beta=0.0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            r = raw.conv1x1_dgrad_wgrad_bnbwd(dy, z, mask, coef, w, y, dw, bn=bn, dw_beta=0.0)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        dx = r[0] if isinstance(r, tuple) else r
        nbytes = 2 * M * K * 2 + M * K // 8 + M * C * 2 * 2 + (M * C * 2 + M * C // 8 if bn else 0)
        out[name] = {
            "ms": round(ms, 4), "TBps": round(nbytes / ms / 1e9, 3), "GB": round(nbytes / 1e9, 3),
            "dx_sum": float(dx.float().sum()), "dx_abs": float(dx.float().abs().sum()),
            "dw_sum": float(dw.sum()), "dw_abs": float(dw.abs().sum()),
        }
        if bn is not None:
            out[name]["stats_sum"] = float(r[1].double().sum())
    # determinism: two launches give the same bits; the statistics epilogue does not change dx
    dw = torch.zeros((K, 1, 1, C), device=dev, dtype=torch.float32)
    r1 = raw.conv1x1_dgrad_wgrad_bnbwd(dy, z, mask, coef, w, y, dw, bn=(z2, m2), dw_beta=0.0)
    r2 = raw.conv1x1_dgrad_wgrad_bnbwd(dy, z, mask, coef, w, y, dw.clone(), bn=(z2, m2), dw_beta=0.0)
    rp = raw.conv1x1_dgrad_wgrad_bnbwd(dy, z, mask, coef, w, y, dw.clone(), dw_beta=0.0)
    out["dx_repeat_equal"] = bool(torch.equal(r1[0], r2[0]))
    out["stats_repeat_equal"] = bool(torch.equal(r1[1], r2[1]))
    out["dx_bn_vs_plain_equal"] = bool(torch.equal(r1[0], rp))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
