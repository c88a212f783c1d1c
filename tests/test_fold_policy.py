"""Which BatchNorm applies the fused ResNet block folds into a 1x1 GEMM (CPU: policy only).

The transform-A core (csrc/include/ca_gemm_xa.h) wins only on long-K, narrow-N GEMMs: on
ResNet-50 that is bn3 -> conv3's input gradient (K = 4c, N = c) and bn3 (+ residual) -> the
next block's conv1 (K = 4c, N = c), in every stage; bn2 -> conv3 and bn1 -> conv1's input
gradient (K = c, N = 4c) stay separate passes (measured: docs/performance.md, round 4).
"""
import pytest

from cloud_amd.models.fused_block import _fold_site

STAGES = (64, 128, 256, 512)  # bottleneck width c of ResNet-50's four stages


@pytest.mark.parametrize("c", STAGES)
def test_long_k_sites_folded(c, monkeypatch):
    monkeypatch.delenv("CLOUD_AMD_BN_FOLD_ALL", raising=False)
    monkeypatch.delenv("CLOUD_AMD_BN_FOLD_MAX_N", raising=False)
    assert _fold_site(4 * c, c)          # bn3 -> conv3 dgrad, bn3 -> next conv1
    assert not _fold_site(c, 4 * c)      # bn2 -> conv3 fwd, bn1 -> conv1 dgrad


def test_knobs(monkeypatch):
    monkeypatch.setenv("CLOUD_AMD_BN_FOLD_MAX_N", "64")
    assert _fold_site(256, 64) and not _fold_site(512, 128)
    monkeypatch.setenv("CLOUD_AMD_BN_FOLD_ALL", "1")
    assert _fold_site(64, 256) and _fold_site(512, 128)
