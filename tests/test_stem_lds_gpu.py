"""LDS-resident space-to-depth stem convolution (csrc/include/ca_conv_stem.h): the ResNet-50 stem
(7x7 / stride 2 / pad 3 over 224 x 224 x 3) as a 4x4 / stride-1 conv over the 16-channel
space-to-depth input, forward with the BN-statistics epilogue, against a plain PyTorch fp32
convolution of the same bf16 operands.  Grids with fewer tiles than workgroups (N = 3: 84 tiles)
and several tiles per workgroup (N = 20: 560 tiles); every partial row must be written and the
rows must sum to the column sums / sums of squares of the stored bf16 output."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b).norm() / b.norm().clamp_min(1e-12))


@pytest.mark.parametrize("N", [3, 20])
def test_stem_lds_forward_matches_fp32_conv(N):
    from cloud_amd.ops import _ext
    from cloud_amd.ops import conv as conv_ops

    ext = _ext.load(required=True)
    torch.manual_seed(100 + N)
    x = torch.randn(N, 224, 224, 3, device="cuda").to(torch.bfloat16)
    w = (torch.randn(64, 7, 7, 8, device="cuda") * 0.1).to(torch.bfloat16)
    assert conv_ops.stem_s2d_ok(x, w, 2, 3)
    rows = ext.conv_stat_rows(N, 115, 115, 16, 64, 4, 4, 1, 1, 0, 0)
    assert rows <= min(N * 28, 256)  # one partial row per persistent workgroup (not per 128 pixels)
    y, part = conv_ops.stem_conv_s2d(x, w, stats=True)
    torch.cuda.synchronize()
    assert part.shape == (rows, 2, 64)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w[..., :3].float().permute(0, 3, 1, 2), stride=2, padding=3)
    ref = ref.permute(0, 2, 3, 1)
    assert y.shape == ref.shape == (N, 112, 112, 64)
    assert _rel(y, ref) < 5e-3
    yf = y.float().reshape(-1, 64)
    assert torch.isfinite(part).all()
    assert _rel(part[:, 0].sum(0), yf.sum(0)) < 1e-3
    assert _rel(part[:, 1].sum(0), (yf * yf).sum(0)) < 1e-3


def test_stem_lds_partials_all_written():
    """Poisoned partials: the kernel must write every row it reports."""
    from cloud_amd.ops import _ext

    ext = _ext.load(required=True)
    N = 5
    torch.manual_seed(7)
    xs = torch.randn(N, 115, 115, 16, device="cuda").to(torch.bfloat16)
    w = (torch.randn(64, 4, 4, 16, device="cuda") * 0.1).to(torch.bfloat16)
    rows = ext.conv_stat_rows(N, 115, 115, 16, 64, 4, 4, 1, 1, 0, 0)
    part = torch.full((rows, 2, 64), float("nan"), device="cuda")
    y = torch.empty(N, 112, 112, 64, device="cuda", dtype=torch.bfloat16)
    ext.conv_fwd(xs.data_ptr(), w.data_ptr(), y.data_ptr(), N, 115, 115, 16, 64, 4, 4, 1, 1, 0, 0, part.data_ptr(),
                 _ext.stream_handle(xs.device))
    torch.cuda.synchronize()
    ref = F.conv2d(xs.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
    assert _rel(y, ref) < 5e-3
    assert torch.isfinite(part).all()
    yf = y.float().reshape(-1, 64)
    assert _rel(part[:, 0].sum(0), yf.sum(0)) < 1e-3
