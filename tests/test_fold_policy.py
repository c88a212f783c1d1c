"""Which BatchNorm applies the fused ResNet block folds into a 1x1 GEMM (CPU: policy only).

The transform-A core (csrc/include/ca_gemm_xa.h) wins only on long-K, narrow-N GEMMs: on
ResNet-50 that is bn3 -> conv3's input gradient (K = 4c, N = c) and bn3 (+ residual) -> the
next block's conv1 (K = 4c, N = c), at stages 1-3 (c <= 256: stage 3 on the two-deep 128 x 256
tiles, round 6; stage 4 measured below stages 1-3 only); bn2 -> conv3 and bn1 -> conv1's input
gradient (K = c, N = 4c) stay separate passes (measured: docs/performance.md, round 4).
"""
import pytest

from cloud_amd.models.fused_block import _fold_site

STAGES = (64, 128, 256, 512)  # bottleneck width c of ResNet-50's four stages


@pytest.mark.parametrize("c", STAGES)
def test_long_k_sites_folded(c, monkeypatch):
    monkeypatch.delenv("CLOUD_AMD_BN_FOLD_ALL", raising=False)
    monkeypatch.delenv("CLOUD_AMD_BN_FOLD_MAX_N", raising=False)
    assert _fold_site(4 * c, c) == (c <= 256)  # bn3 -> conv3 dgrad, bn3 -> next conv1
    assert not _fold_site(c, 4 * c)            # bn2 -> conv3 fwd, bn1 -> conv1 dgrad


def test_knobs(monkeypatch):
    monkeypatch.setenv("CLOUD_AMD_BN_FOLD_MAX_N", "64")
    assert _fold_site(256, 64) and not _fold_site(512, 128)
    monkeypatch.setenv("CLOUD_AMD_BN_FOLD_MAX_N", "4096")
    assert _fold_site(2048, 512) and _fold_site(1024, 256)
    monkeypatch.setenv("CLOUD_AMD_BN_FOLD_ALL", "1")
    assert _fold_site(64, 256) and _fold_site(512, 128)


def test_fused_weight_gradient_shapes():
    """One-pass input + weight gradient (ca_gemm_xa_dw): the dW block must fit the
    registers of a workgroup -- stage-1 conv3 (K 256 -> N 64) and conv1 (K 64 -> N 256) with
    4 waves, stage-2 conv3 (K 512 -> N 128) with 8 waves; nothing wider."""
    from cloud_amd.ops.raw import dgrad_wgrad_fusable

    assert dgrad_wgrad_fusable(256, 64) and dgrad_wgrad_fusable(64, 256) and dgrad_wgrad_fusable(64, 64)
    assert dgrad_wgrad_fusable(512, 128)
    assert not dgrad_wgrad_fusable(1024, 256) and not dgrad_wgrad_fusable(128, 512)
    assert not dgrad_wgrad_fusable(2048, 512) and not dgrad_wgrad_fusable(256, 1024)
