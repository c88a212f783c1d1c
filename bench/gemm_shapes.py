#!/usr/bin/env python3
"""Micro-benchmark of the ResNet-50 1x1-convolution GEMMs (bs=256, NHWC, bf16).

For every distinct (M, K, N) it times forward ``Y = X W^T``, dgrad ``dX = dY W``
and wgrad ``dW = dY^T X`` through hipBLASLt (torch.mm) and, for wgrad, split-K
variants; when the cloud_amd extension provides MFMA GEMM kernels they are
timed too.  Prints one JSON line per shape.
"""
import json
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    return s.elapsed_time(e) / iters * 1000.0  # us


def shapes(batch=256):
    out = []
    hw = 56
    cin = 64
    for n, w in zip((3, 4, 6, 3), (64, 128, 256, 512)):
        for j in range(n):
            stride = 2 if (j == 0 and w != 64) else 1
            hw_out = hw // stride
            M_in, M_out = batch * hw * hw, batch * hw_out * hw_out
            # conv1 (1x1 cin->w) at input res (stride on 3x3 in v1.5)
            out.append((M_in, cin, w))
            out.append((M_out, w, 4 * w))       # conv3
            if j == 0:
                out.append((M_out, cin, 4 * w))  # downsample (after stride gather)
            cin = 4 * w
            hw = hw_out
    uniq = sorted(set(out), key=lambda t: -t[0] * t[1] * t[2])
    return out, uniq


def main():
    dev = "cuda"
    allshapes, uniq = shapes()
    counts = {s: allshapes.count(s) for s in uniq}
    ext = None
    try:
        from cloud_amd.ops import gemm as cg

        ext = cg
    except Exception:
        pass
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0, "wgrad_best": 0.0}
    for (M, K, N) in uniq:
        X = torch.randn(M, K, device=dev).to(torch.bfloat16)
        W = torch.randn(N, K, device=dev).to(torch.bfloat16)
        dY = torch.randn(M, N, device=dev).to(torch.bfloat16)
        r = {"M": M, "K": K, "N": N, "count": counts[(M, K, N)]}
        r["fwd"] = timeit(lambda: torch.mm(X, W.t()))
        r["dgrad"] = timeit(lambda: torch.mm(dY, W))
        r["wgrad"] = timeit(lambda: torch.mm(dY.t(), X))
        best = r["wgrad"]
        for S in (4, 8, 16, 32, 64):
            if M % S:
                continue
            a = dY.view(S, M // S, N).transpose(1, 2)
            b = X.view(S, M // S, K)
            t = timeit(lambda: torch.bmm(a, b).sum(0, dtype=torch.float32))
            r[f"wgrad_bmm{S}"] = t
            best = min(best, t)
        if ext is not None:
            r["ca_fwd"] = timeit(lambda: ext.mm_nt(X, W))
            r["ca_dgrad"] = timeit(lambda: ext.mm_nn(dY, W))
            out = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
            r["ca_wgrad"] = timeit(lambda: ext.mm_tn_into(dY, X, out))
            for k in ("ca_fwd", "ca_dgrad", "ca_wgrad"):
                tot.setdefault(k, 0.0)
                tot[k] += r[k] * counts[(M, K, N)]
        flops = 2.0 * M * K * N
        r["fwd_TF"] = flops / r["fwd"] / 1e6
        r["wgrad_best"] = best
        for k in ("fwd", "dgrad", "wgrad", "wgrad_best"):
            tot[k] += r[k] * counts[(M, K, N)]
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
        del X, W, dY
    print(json.dumps({"total_ms": {k: round(v / 1000, 3) for k, v in tot.items()}}))


if __name__ == "__main__":
    main()
