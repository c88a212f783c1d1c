"""Fused ResNet stem tail (BN + ReLU + 3x3/2 max-pool forward; max-pool backward fused with
the BN-backward statistics) against the separate native ops it replaces, and against an
fp32 PyTorch reference."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("N,H,W", [(2, 32, 32), (3, 33, 29), (2, 112, 112)])
def test_stem_tail_matches_separate_ops(N, H, W):
    from cloud_amd.models.layers import BatchNormAct, MaxPool2d
    from cloud_amd.ops import _ext, gemm
    from cloud_amd.ops.pooling import stem_bn_relu_maxpool, stem_tail_ok

    _ext.load(required=True)
    torch.manual_seed(N * H + W)
    C = 64
    z0 = (torch.randn(N, H, W, C, device=DEV) * 2 + 0.3).to(torch.bfloat16)
    M = N * H * W
    part = torch.empty(((M + 127) // 128, 2, C), device=DEV)
    gemm.fill_stats_torch(z0.view(M, C), part)
    bns = [BatchNormAct(C, relu=True, device=DEV) for _ in range(2)]
    gamma, beta = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.2
    with torch.no_grad():
        for b in bns:  # both sides share one gamma / beta
            b.weight.copy_(gamma)
            b.bias.copy_(beta)
    pool = MaxPool2d(3, 2, 1)
    za = z0.clone().requires_grad_()
    assert stem_tail_ok(za, bns[0], pool, part)
    ya = stem_bn_relu_maxpool(za, bns[0], part)
    zb = z0.clone().requires_grad_()
    yb = pool(bns[1]((zb, part)))
    # same statistics; the apply arithmetic may differ in the last fp32 bit before the bf16
    # rounding (scale/shift FMA vs normalise-then-affine): at most 1 bf16 ulp, rarely
    d = (ya.float() - yb.float()).abs()
    assert float(d.max()) <= 1e-2 * float(yb.float().abs().max()) + 1e-6, float(d.max())
    assert float((d > 0).float().mean()) < 1e-2, float((d > 0).float().mean())
    dy = torch.randn_like(ya)
    ya.backward(dy)
    yb.backward(dy)
    torch.testing.assert_close(za.grad.float(), zb.grad.float(), atol=2e-2, rtol=2e-2)
    for pa, pb in ((bns[0].weight, bns[1].weight), (bns[0].bias, bns[1].bias)):
        torch.testing.assert_close(pa.grad, pb.grad, atol=1e-2, rtol=1e-3)
    torch.testing.assert_close(bns[0].running_mean, bns[1].running_mean)
    torch.testing.assert_close(bns[0].running_var, bns[1].running_var)
    # fp32 reference of the whole tail
    zr = z0.float().requires_grad_()
    w = bns[0].weight.detach().clone().requires_grad_()
    b = bns[0].bias.detach().clone().requires_grad_()
    mean = zr.mean((0, 1, 2))
    var = zr.var((0, 1, 2), unbiased=False)
    yr = torch.relu((zr - mean) * torch.rsqrt(var + 1e-5) * w + b)
    yr = F.max_pool2d(yr.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    torch.testing.assert_close(ya.float(), yr, atol=3e-2, rtol=2e-2)
    yr.backward(dy.float())
    # bf16-rounded BN outputs tie inside pooling windows where fp32 does not, so some window
    # gradients land on a different pixel (the separate bf16 ops do the same): 2-3 % here
    err = (za.grad.float() - zr.grad).norm() / zr.grad.norm()
    assert float(err) < 5e-2, float(err)
    for ours, ref in ((bns[0].weight.grad, w.grad), (bns[0].bias.grad, b.grad)):
        rel = (ours - ref).norm() / ref.norm()  # same tie routing: single channels move a few %
        assert float(rel) < 2e-2, float(rel)
