"""Persistent resident-weight GEMM core (csrc/include/ca_gemm_prw.h) for the small-K forward
1x1 convolutions with the BN-statistics epilogue, against a plain PyTorch fp32 GEMM of the
same bf16 operands: every covered (N, K), a ragged last tile, grids with fewer tiles than
workgroups and many tiles per workgroup; the [rows][2][N] partials (one row per workgroup,
or per row range for the column-chunked kinds -- ResNet's conv3 expansions, N = 512..2048)
must sum to the column sums / sums of squares of the stored bf16 output.  Also checks that
the fused ResNet block's forward statistics agree with and without the core."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b).norm() / b.norm().clamp_min(1e-12))


PERSISTENT = {(256, 64), (512, 128), (1024, 256)}


@pytest.mark.parametrize("N,K", [(256, 64), (64, 64), (64, 256), (128, 256), (512, 128), (1024, 256),
                                 (2048, 512)])
@pytest.mark.parametrize("M", [128 * 3 + 17, 128 * 8 + 5, 200_000 + 77])
def test_prw_forward_stats(N, K, M):
    """PERSISTENT shapes run on the persistent core (column-chunked above N = 256, when the grid
    has at least 8 row ranges); the other shapes check that the row count the host reports
    matches what the tiled core writes."""
    from cloud_amd.ops import _ext, raw

    ext = _ext.load(required=True)
    torch.manual_seed(N + K + M)
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    st = raw.gemm_stats_buffer(M, N, K, a.device)
    rows = ext.gemm_stat_rows(M, N, K, K, K, N)
    assert st.shape == (rows, 2, N)
    assert rows <= (M + 127) // 128  # persistent: one row per workgroup (<= one per tile)
    if (N, K) not in PERSISTENT:
        assert rows == (M + 127) // 128
    st.fill_(float("nan"))  # every row must be written
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ext.gemm_bf16(raw.NT, a.data_ptr(), K, w.data_ptr(), K, y.data_ptr(), N, M, N, K, st.data_ptr(), 0.0,
                  _ext.stream_handle(a.device))
    torch.cuda.synchronize()
    ref = a.float() @ w.float().t()
    assert _rel(y, ref) < 5e-3
    yf = y.float()
    assert torch.isfinite(st).all()
    assert _rel(st[:, 0].sum(0), yf.sum(0)) < 1e-3
    assert _rel(st[:, 1].sum(0), (yf * yf).sum(0)) < 1e-3


def test_prw_rows_fall_back_when_not_covered():
    from cloud_amd.ops import _ext

    ext = _ext.load(required=True)
    M = 50_000
    # K = 512 (weight too large to stay resident): tiled core, one row per 128 GEMM rows
    assert ext.gemm_stat_rows(M, 128, 512, 512, 512, 128) == (M + 127) // 128
    # covered shape: at most (workgroups per CU) x CUs rows
    assert ext.gemm_stat_rows(M, 256, 64, 64, 64, 256) <= 4 * 256
    # column-chunked kinds: one row per range of row tiles (8 ranges per XCD or fewer)
    assert ext.gemm_stat_rows(M, 1024, 256, 256, 256, 1024) in (32, (M + 127) // 128)
    # too few tiles for 8 ranges: tiled core
    assert ext.gemm_stat_rows(500, 1024, 256, 256, 256, 1024) == 4


def test_conv_fwd_1x1_stats_match_tiled_core():
    """raw.conv_fwd + conv_stats_buffer (the fused block's forward path) on a ResNet stage-1
    conv3 shape: the partials sum to the same column statistics as the output."""
    from cloud_amd.ops import raw

    torch.manual_seed(11)
    x = torch.randn(8, 56, 56, 64, device="cuda").to(torch.bfloat16)
    w = (torch.randn(256, 1, 1, 64, device="cuda") * 0.1).to(torch.bfloat16)
    part = raw.conv_stats_buffer(x.shape, w, 1, 0, x.device)
    y = raw.conv_fwd(x, w, 1, 0, stats=part)
    ref = x.float().reshape(-1, 64) @ w.float().reshape(256, 64).t()
    assert _rel(y.reshape(-1, 256), ref) < 5e-3
    yf = y.float().reshape(-1, 256)
    assert _rel(part[:, 0].sum(0), yf.sum(0)) < 1e-3
    assert _rel(part[:, 1].sum(0), (yf * yf).sum(0)) < 1e-3
