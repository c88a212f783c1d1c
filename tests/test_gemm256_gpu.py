"""The 256 x 256 GEMM cores -- the ring core (csrc/include/ca_gemm256.h, core kind 4 = v256)
and the 8-phase core (csrc/include/ca_gemm256p8.h, core kind 6 = vp8), each forced on every
GEMM with M, N >= 256 -- against a plain PyTorch fp32
GEMM of the same bf16 operands: forward (NT), input grad (NN), weight grad (TN, split-K fp32
slabs), the fused bias + activation and BN-statistics epilogues, ragged M / N / K (partial
tiles, K tails read as zeros through the buffer range check), one to many K tiles -- plus
the default dispatch (core kind 3) on a shape that selects the 256 core by itself."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(params=[4, 6], ids=["ring256", "p8"])
def core256(request):
    """Force a 256 x 256 core on every GEMM with M, N >= 256: 4 = the ring core (v256),
    6 = the 8-phase core (vp8, csrc/include/ca_gemm256p8.h)."""
    from cloud_amd.ops import _ext

    ext = _ext.load(required=True)
    if request.param == 4 and not ext.experimental_built():
        pytest.skip("ring core: experiment-only, built with CLOUD_AMD_BUILD_EXPERIMENTAL=1")
    prev = ext.gemm_set_core(request.param)
    assert prev >= 0
    yield request.param
    ext.gemm_set_core(prev)


def _rel(a, b):
    return float((a.float() - b).norm() / b.norm())


@pytest.mark.parametrize("M,N,K", [(512, 512, 64), (1024, 768, 2048), (300, 264, 200), (4096, 256, 1024),
                                   (777, 1032, 4104)])
def test_256_forward_and_input_grad(core256, M, N, K):
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
def test_256_weight_grad_splitk(core256, M, N, K):
    from cloud_amd.ops import raw

    torch.manual_seed(M + N)
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    gw = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
    raw.wgrad_into(dy, x, gw, beta=0.0)
    assert _rel(gw, dy.float().t() @ x.float()) < 5e-3


def test_256_bias_act_and_stats_epilogues(core256):
    from cloud_amd.ops import raw

    torch.manual_seed(7)
    M, N, K = 1024, 512, 320
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    bias = torch.randn(N, device="cuda")
    ref = a.float() @ w.float().t() + bias
    y = raw.gemm(a, w, bias=bias, act="relu")
    assert _rel(y, torch.relu(ref)) < 5e-3
    st = raw.stats_buffer(M, N, a.device)
    y2 = raw.gemm(a, w, stats=st)
    z = (a.float() @ w.float().t())
    s_sum = st.view(-1, 2, N)[:, 0].sum(0)
    s_sq = st.view(-1, 2, N)[:, 1].sum(0)
    assert _rel(y2, z) < 5e-3
    assert _rel(s_sum, y2.float().sum(0)) < 1e-3
    assert _rel(s_sq, (y2.float() ** 2).sum(0)) < 1e-3


def test_default_dispatch_selects_256_on_large_gemm():
    """8192 x 2048 x 1024: 256 tiles of 256 x 256 (one full round), 32 K tiles -> the default
    dispatch (kind 5) uses the two-phase 256 core; result checked against fp32."""
    from cloud_amd.ops import _ext, raw

    ext = _ext.load(required=True)
    prev = ext.gemm_set_core(5)
    try:
        torch.manual_seed(3)
        a = torch.randn(8192, 1024, device="cuda").to(torch.bfloat16)
        w = torch.randn(2048, 1024, device="cuda").to(torch.bfloat16)
        y = raw.gemm(a, w)
        assert _rel(y[:1024], a[:1024].float() @ w.float().t()) < 5e-3
    finally:
        ext.gemm_set_core(prev)


@pytest.mark.parametrize("M,N,K", [(8192, 3072, 768), (8000, 1000, 704), (4096, 2048, 4096)])
def test_256x128_core_dispatch(M, N, K, monkeypatch):
    """The 256 x 128 single-phase core (ca_gemm256p8.h mfma_gemm_256x128, opt-in with
    CLOUD_AMD_GEMM_256X128=1, read once per process -- so this test also covers whatever the
    process decided) where 256 x 128 tiles fill whole rounds (BERT FFN1 forward / FFN2 input
    gradient shape first; ragged M / N / K): forward with bias + GELU + pre-activation, input
    gradient with GELU' -- against fp32 references."""
    from cloud_amd.ops import _ext, raw

    if not _ext.load(required=True).experimental_built():
        pytest.skip("256 x 128 core: experiment-only, built with CLOUD_AMD_BUILD_EXPERIMENTAL=1")
    monkeypatch.setenv("CLOUD_AMD_GEMM_256X128", "1")

    torch.manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device="cuda") * 0.1
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    y = raw.gemm(a, w, bias=b, act="gelu", preact=pre)
    ref = a.float() @ w.float().t() + b
    assert _rel(pre, ref) < 5e-3
    assert _rel(y, torch.nn.functional.gelu(pre.float())) < 1e-2
    w2 = (torch.randn(K, N, device="cuda") * 0.05).to(torch.bfloat16)  # NN: dx[M, N] = dy[M, K] @ w2[K, N]
    dy = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    dx = raw.gemm(dy, w2, layout=raw.NN, act="gelu", dact_src=pre)
    ref2 = (dy.float() @ w2.float()) * _gelu_grad(pre.float())
    assert _rel(dx, ref2) < 1e-2, _rel(dx, ref2)


def _gelu_grad(x):
    cdf = 0.5 * (1.0 + torch.erf(x / 2 ** 0.5))
    pdf = torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5
    return cdf + x * pdf
