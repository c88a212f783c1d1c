"""256 x 96 forward GEMM tiles (csrc/kernels/gemm.hip use_256x96 / dense_gemm_256x96_kernel),
taken when the 96-wide grid fills whole rounds of the chip and the 128 x 128 grid does not --
BERT-base's QKV projection (M = 8192, N = 2304, K = 768).  Against plain PyTorch fp32 GEMMs of
the same bf16 operands: plain, bias, bias + GELU with the kept pre-activation; bitwise
run-to-run."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b).norm() / b.norm())


@pytest.mark.parametrize("bias,act", [(False, None), (True, None), (True, "gelu")])
def test_qkv_shape_forward(bias, act):
    from cloud_amd.ops import raw

    torch.manual_seed(11)
    M, N, K = 8192, 2304, 768
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda") if bias else None
    kw = {}
    if act:
        kw = dict(act=act, preact=torch.empty(M, N, device="cuda", dtype=torch.bfloat16))
    y = raw.gemm(x, w, bias=b, **kw)
    ref = x.float() @ w.float().t() + (b if bias else 0)
    if act:
        assert _rel(kw["preact"], ref) < 5e-3
        ref = torch.nn.functional.gelu(ref)
    assert _rel(y, ref) < 8e-3
    again = raw.gemm(x, w, bias=b, **kw)
    assert torch.equal(again, y)
