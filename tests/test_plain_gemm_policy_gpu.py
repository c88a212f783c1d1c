"""Plain-GEMM engine policy (ops/raw.py PlainGemmPolicy, CLOUD_AMD_GEMM_LIB): in every mode a
plain GEMM -- NT with bias, NN with C accumulate -- matches a plain PyTorch fp32 GEMM of the
same bf16 operands; ``auto`` records one timed decision per shape; fused GEMMs (activation,
pre-activation, act') never leave the in-tree kernels."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b).norm() / b.norm())


@pytest.mark.parametrize("mode", ["never", "always", "auto"])
def test_plain_gemm_modes_match_fp32(mode):
    from cloud_amd.ops import raw

    pol = raw.PLAIN_GEMM
    prev_mode, prev_dec = pol.mode, dict(pol.decisions)
    pol.mode, pol.decisions = mode, {}
    try:
        torch.manual_seed(5)
        a = torch.randn(1024, 768, device="cuda").to(torch.bfloat16)
        w = (torch.randn(2304, 768, device="cuda") * 0.05).to(torch.bfloat16)
        b = torch.randn(2304, device="cuda")
        y = raw.gemm(a, w, bias=b)
        assert _rel(y, a.float() @ w.float().t() + b) < 5e-3
        g = torch.randn(1024, 2304, device="cuda").to(torch.bfloat16)
        acc = torch.randn(1024, 768, device="cuda").to(torch.bfloat16)
        ref = acc.float() + g.float() @ w.float()
        raw.gemm(g, w, layout=raw.NN, out=acc, beta=1.0)
        assert _rel(acc, ref) < 5e-3
        if mode == "auto":
            assert len(pol.decisions) == 2
            assert all({"library", "ours_us", "lib_us"} <= set(d) for d in pol.decisions.values())
        # fused: bias + GELU with the pre-activation kept never goes to the library
        pre = torch.empty_like(y)
        n_dec = len(pol.decisions)
        f = raw.gemm(a, w, bias=b, act="gelu", preact=pre)
        assert len(pol.decisions) == n_dec
        assert _rel(pre, a.float() @ w.float().t() + b) < 5e-3
        assert _rel(f, torch.nn.functional.gelu(pre.float())) < 1e-2
    finally:
        pol.mode, pol.decisions = prev_mode, prev_dec
