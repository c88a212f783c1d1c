"""Flattened-halo 3x3 / stride-1 forward convolution (conv.hip conv3x3_halo_kernel, opt-in via
CLOUD_AMD_CONV_HALO=1, read once per process) against an fp32 PyTorch reference.  Runs in a
child process so the switch is on for that process only."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, torch, torch.nn.functional as F
sys.path.insert(0, sys.argv[1])
from cloud_amd.ops import raw
torch.manual_seed(3)
# (N, H, Cin, Cout): 64-wide tiles, 2 channel chunks x 128-wide tiles with a partial second
# N tile, a 7x7 map (every tile row touches a border), halo rows past the last image
for N, H, cin, cout in [(2, 14, 64, 64), (3, 7, 128, 192), (1, 56, 64, 64), (2, 28, 128, 128)]:
    x = torch.randn(N, H, H, cin, device="cuda").to(torch.bfloat16)
    w = (torch.randn(cout, 3, 3, cin, device="cuda") / (9 * cin) ** 0.5).to(torch.bfloat16)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), None, 1, 1).permute(0, 2, 3, 1)
    y = raw.conv_fwd(x, w, 1, 1)
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)
    st = raw.stats_buffer(N * H * H, cout, x.device)
    y2 = raw.conv_fwd(x, w, 1, 1, stats=st)
    torch.testing.assert_close(y2.float(), ref, atol=3e-2, rtol=3e-2)
    yf = y2.float().reshape(-1, cout)
    torch.testing.assert_close(st[:, 0].sum(0), yf.sum(0), atol=1e-1, rtol=1e-3)
    torch.testing.assert_close(st[:, 1].sum(0), (yf * yf).sum(0), atol=1e-1, rtol=1e-3)
print("halo ok")
"""


@pytest.mark.gpu
def test_conv3x3_halo_matches_fp32():
    env = dict(os.environ, CLOUD_AMD_CONV_HALO="1")
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "halo ok" in r.stdout
