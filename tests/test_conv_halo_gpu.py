"""The LDS-resident 3x3 convolution (csrc/include/ca_conv_halo.h): ResNet-50 stage-1 conv2
(3x3, stride 1, pad 1, 64 -> 64 channels, 56 x 56) forward with the BN-forward statistics
epilogue and input gradient with the BN-backward statistics epilogue, against plain PyTorch fp32
convolutions of the same bf16 operands.  Batch 4 runs one tile per workgroup; batch 64 runs
448 tiles on the persistent grid (several tiles per workgroup, the next patch prefetched)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b).norm() / b.norm())


def _nchw(t):
    return t.float().permute(0, 3, 1, 2)


@pytest.mark.parametrize("N", [4, 64])
def test_halo_forward_with_statistics(N):
    from cloud_amd.ops import raw

    torch.manual_seed(N)
    x = torch.randn(N, 56, 56, 64, device="cuda").to(torch.bfloat16)
    w = (torch.randn(64, 3, 3, 64, device="cuda") / 24).to(torch.bfloat16)
    part = raw.conv_stats_buffer(x.shape, w, 1, 1, x.device)
    y = raw.conv_fwd(x, w, 1, 1, stats=part)
    ref = F.conv2d(_nchw(x), _nchw(w), padding=1).permute(0, 2, 3, 1)
    assert _rel(y, ref) < 5e-3
    yf = y.float().reshape(-1, 64)
    s, q = part[:, 0].sum(0), part[:, 1].sum(0)
    torch.testing.assert_close(s, yf.sum(0), rtol=1e-3, atol=1e-1)
    torch.testing.assert_close(q, (yf * yf).sum(0), rtol=1e-3, atol=1e-1)


@pytest.mark.parametrize("N", [4, 64])
def test_halo_input_gradient_with_bn_statistics(N):
    from cloud_amd.ops import raw

    torch.manual_seed(100 + N)
    dy = torch.randn(N, 56, 56, 64, device="cuda").to(torch.bfloat16)
    w = (torch.randn(64, 3, 3, 64, device="cuda") / 24).to(torch.bfloat16)
    z = torch.randn(N, 56, 56, 64, device="cuda").to(torch.bfloat16)
    mask = torch.randint(0, 256, (N * 56 * 56, 8), device="cuda", dtype=torch.uint8)
    dx, part = raw.conv_dgrad(dy, w, (N, 56, 56, 64), 1, 1, bn=(z, mask))
    ref = F.conv_transpose2d(_nchw(dy), _nchw(w).contiguous(), padding=1).permute(0, 2, 3, 1)
    assert _rel(dx, ref) < 5e-3
    bits = ((mask.long().unsqueeze(-1) >> torch.arange(8, device="cuda")) & 1).reshape(-1, 64).float()
    g = dx.float().reshape(-1, 64) * bits
    torch.testing.assert_close(part[:, 0].sum(0), g.sum(0), rtol=1e-3, atol=1e-1)
    torch.testing.assert_close(part[:, 1].sum(0), (g * z.float().reshape(-1, 64)).sum(0), rtol=1e-3, atol=1e-1)


def test_halo_plain_input_gradient_and_forward_without_statistics():
    from cloud_amd.ops import raw

    torch.manual_seed(5)
    x = torch.randn(8, 56, 56, 64, device="cuda").to(torch.bfloat16)
    w = (torch.randn(64, 3, 3, 64, device="cuda") / 24).to(torch.bfloat16)
    y = raw.conv_fwd(x, w, 1, 1)
    assert _rel(y, F.conv2d(_nchw(x), _nchw(w), padding=1).permute(0, 2, 3, 1)) < 5e-3
    dx = raw.conv_dgrad(y, w, x.shape, 1, 1)
    ref = F.conv_transpose2d(_nchw(y), _nchw(w).contiguous(), padding=1).permute(0, 2, 3, 1)
    assert _rel(dx, ref) < 5e-3


@pytest.mark.parametrize("N", [4, 64])
def test_halo_weight_gradient(N):
    """conv3x3_halo_wgrad: one fp32 [64][576] partial per persistent workgroup, split-K reduce
    into the bf16 gradient with beta accumulation (the flat-arena contract)."""
    from cloud_amd.ops import raw

    torch.manual_seed(200 + N)
    x = torch.randn(N, 56, 56, 64, device="cuda").to(torch.bfloat16)
    dy = torch.randn(N, 56, 56, 64, device="cuda").to(torch.bfloat16)
    prev = (torch.randn(64, 3, 3, 64, device="cuda") * 10).to(torch.bfloat16)
    out = prev.clone()
    raw.conv_wgrad(dy, x, (64, 3, 3, 64), 1, 1, out=out, beta=1.0)
    ref = torch.nn.grad.conv2d_weight(_nchw(x), (64, 64, 3, 3), _nchw(dy), padding=1).permute(0, 2, 3, 1)
    assert _rel(out.float() - prev.float(), ref) < 2e-2  # bf16 output rounding on top of the sum
    out32 = torch.zeros(64, 3, 3, 64, device="cuda")
    raw.conv_wgrad(dy, x, (64, 3, 3, 64), 1, 1, out=out32, beta=0.0)
    assert _rel(out32, ref) < 2e-3
