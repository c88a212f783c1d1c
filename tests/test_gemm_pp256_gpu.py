"""The opt-in 256 x 256 ping-pong GEMM core (csrc/include/ca_mfma_core.h mfma_gemm_pp256,
CLOUD_AMD_GEMM_CORE=pp256) against a plain PyTorch fp32 GEMM of the same bf16 operands:
forward (NT), input grad (NN), weight grad (TN, split-K fp32 slabs), ragged M / N / K
(partial tiles, the zero page for K beyond the end), one and several K tiles."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def pp256():
    from cloud_amd.ops import _ext

    ext = _ext.load(required=True)
    prev = ext.gemm_set_core(4)
    yield
    ext.gemm_set_core(prev)


def _rel(a, b):
    return float((a.float() - b).norm() / b.norm())


@pytest.mark.parametrize("M,N,K", [(512, 512, 64), (1024, 768, 2048), (300, 264, 200), (4096, 256, 1024),
                                   (777, 1032, 4104)])
def test_pp256_forward_and_input_grad(pp256, M, N, K):
    from cloud_amd.ops import raw

    torch.manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    y = raw.gemm(a, w)
    assert _rel(y, a.float() @ w.float().t()) < 5e-3
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    dx = raw.gemm(dy, w, layout=raw.NN)
    assert _rel(dx, dy.float() @ w.float()) < 5e-3


@pytest.mark.parametrize("M,N,K", [(8192, 512, 256), (2000, 1024, 512)])
def test_pp256_weight_grad_splitk(pp256, M, N, K):
    from cloud_amd.ops import raw

    torch.manual_seed(M + N)
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    gw = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
    raw.wgrad_into(dy, x, gw, beta=0.0)
    assert _rel(gw, dy.float().t() @ x.float()) < 5e-3
