"""HBM bandwidth of the training BatchNorm apply passes on the ResNet-50 b1024 shapes.

Forward: bn_fwd from epilogue partials (finalize + apply: read z [+ residual], write y and
the ReLU bitmask).  Backward: bn_bwd from epilogue partials (finalize + apply: read dy, z
and the bitmask, write dz).  Time per call from HIP events (the finalize is a ~5 us
per-channel kernel included in the time); bytes are the apply pass's minimum traffic.

usage: [CLOUD_AMD_BN_APPLY_BLOCKS=N] python bench/bn_apply_bw.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloud_amd.ops import raw  # noqa: E402

SHAPES = [  # rows M (= N*H*W at batch 1024), channels C
    (3211264, 64), (3211264, 256), (802816, 128), (802816, 512), (200704, 256), (200704, 1024),
    (50176, 512), (50176, 2048),
]


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    torch.manual_seed(0)
    dev = torch.device("cuda")
    blocks = os.environ.get("CLOUD_AMD_BN_APPLY_BLOCKS", "0") + "/ilv" + os.environ.get("CLOUD_AMD_BN_APPLY_ILV", "1")
    for M, C in SHAPES:
        z = torch.randn(M, C, device=dev).to(torch.bfloat16)
        g = torch.randn(M, C, device=dev).to(torch.bfloat16)
        res = torch.randn(M, C, device=dev).to(torch.bfloat16)
        gamma = torch.rand(C, device=dev) + 0.5
        beta = torch.randn(C, device=dev) * 0.1
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        zf = z.float()
        parts = torch.stack([zf.sum(0), (zf * zf).sum(0)]).unsqueeze(0).contiguous()
        y, stats, mask = raw.bn_fwd(z, gamma, beta, rm, rv, 1e-5, 0.0, True, partials=parts, keep_mask=True)
        # numerics vs fp32: y = relu(gamma * (z - mean) * rstd + beta), and the bitmask
        mean, var = zf.mean(0), zf.var(0, unbiased=False)
        ref = torch.relu(gamma * (zf - mean) * torch.rsqrt(var + 1e-5) + beta)
        err = float((y.float() - ref).norm() / ref.norm())
        assert err < 1e-2, err
        bits = (ref.view(M, C // 8, 8) > 0).to(torch.int32) << torch.arange(8, device=dev, dtype=torch.int32)
        mask_ok = float((bits.sum(-1).to(torch.uint8) == mask).float().mean())
        gp = torch.stack([g.float().sum(0), (g.float() * zf).sum(0)]).unsqueeze(0).contiguous()
        dgam, dbet = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        nb = M * C * 2
        t_fwd = timeit(lambda: raw.bn_fwd(z, gamma, beta, rm, rv, 1e-5, 0.0, True, partials=parts, keep_mask=True))
        t_res = timeit(lambda: raw.bn_fwd(z, gamma, beta, rm, rv, 1e-5, 0.0, True, residual=res, partials=parts,
                                          keep_mask=True))
        dx = torch.empty_like(z)
        t_copy = timeit(lambda: dx.copy_(z))
        t_bwd = timeit(lambda: raw.bn_bwd(g, None, z, gamma, stats, True, dgam, dbet, mask=mask, partials=gp,
                                          dx_out=dx))
        print(json.dumps({
            "M": M, "C": C, "apply_blocks": blocks, "fwd_rel_err": round(err, 5), "mask_match": mask_ok,
            "copy_TBs": round(nb * 2 / t_copy / 1e6, 2), "fwd_us": round(t_fwd, 1), "fwd_TBs": round(nb * (2 + 1 / 16) / t_fwd / 1e6, 2),
            "fwd_res_us": round(t_res, 1), "fwd_res_TBs": round(nb * (3 + 1 / 16) / t_res / 1e6, 2),
            "bwd_us": round(t_bwd, 1), "bwd_TBs": round(nb * (3 + 1 / 16) / t_bwd / 1e6, 2)}), flush=True)
        del z, g, res, y, mask, dx, zf, ref, bits


if __name__ == "__main__":
    main()
