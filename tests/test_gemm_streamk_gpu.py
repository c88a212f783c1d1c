"""Stream-K GEMM (csrc/include/ca_gemm256p8.h mfma_gemm_256p8_sk): one workgroup per CU over
all (256 x 256 tile, K iteration) pairs; a tile split across workgroups is finished by its
owner, which adds the other contributors' fp32 partial tiles in a fixed order behind an
agent-scope ticket.  Against plain PyTorch fp32 GEMMs of the same bf16 operands: forward (NT)
and input gradient (NN), ragged M / N / K, tiles shared by one to many workgroups, the dense
layer's bias + GELU + pre-activation epilogue and the GELU' input-gradient epilogue at BERT's
shapes; bitwise run-to-run (the partial sum order is fixed); many launches back to back (the
owners leave every ticket at zero for the next launch)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def streamk():
    from cloud_amd.ops import _ext

    ext = _ext.load(required=True)
    if not ext.experimental_built():
        pytest.skip("stream-K: experiment-only, built with CLOUD_AMD_BUILD_EXPERIMENTAL=1")
    prev = ext.gemm_set_streamk(2)  # wherever the operands allow
    yield ext
    ext.gemm_set_streamk(prev)


def _rel(a, b):
    return float((a.float() - b).norm() / b.norm())


@pytest.mark.parametrize("M,N,K", [(512, 512, 128), (1000, 776, 600), (8192, 768, 3072), (300, 264, 4104),
                                   (2048, 2048, 128), (4096, 1024, 8192)])
def test_streamk_forward_and_input_grad(streamk, M, N, K):
    from cloud_amd.ops import raw

    torch.manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    y = raw.gemm(a, w)
    assert _rel(y, a.float() @ w.float().t()) < 5e-3
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    dx = raw.gemm(dy, w, layout=raw.NN)
    assert _rel(dx, dy.float() @ w.float()) < 5e-3


def test_streamk_bitwise_run_to_run_and_back_to_back(streamk):
    from cloud_amd.ops import raw

    torch.manual_seed(3)
    a = torch.randn(8192, 768, device="cuda").to(torch.bfloat16)
    w = torch.randn(2304, 768, device="cuda").to(torch.bfloat16)
    ref = raw.gemm(a, w)
    outs = [raw.gemm(a, w) for _ in range(40)]
    torch.cuda.synchronize()
    assert all(torch.equal(o, ref) for o in outs)
    assert _rel(ref, a.float() @ w.float().t()) < 5e-3


@pytest.mark.parametrize("N,K", [(2304, 768), (3072, 768), (768, 3072), (768, 768)])
def test_streamk_bert_dense_epilogues(N, K):
    """Auto mode on BERT-base's M = 8192 shapes: forward with bias + GELU + kept
    pre-activation, input gradient with GELU' from the pre-activation."""
    from cloud_amd.ops import _ext, raw

    ext = _ext.load(required=True)
    prev = ext.gemm_set_streamk(1)
    try:
        torch.manual_seed(N + K)
        M = 8192
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
        b = torch.randn(N, device="cuda")
        pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        y = raw.gemm(x, w, bias=b, act="gelu", preact=pre)
        ref_pre = x.float() @ w.float().t() + b
        assert _rel(pre, ref_pre) < 5e-3
        assert _rel(y, torch.nn.functional.gelu(ref_pre)) < 8e-3
        dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        pre_k = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        dx = raw.gemm(dy, w, layout=raw.NN, dact_src=pre_k, act="gelu")
        p = pre_k.float()
        dgelu = 0.5 * (1 + torch.erf(p * 0.7071067811865476)) + p * 0.3989422804014327 * torch.exp(-0.5 * p * p)
        assert _rel(dx, (dy.float() @ w.float()) * dgelu) < 8e-3
    finally:
        ext.gemm_set_streamk(prev)
