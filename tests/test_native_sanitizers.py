"""Host-side native code under sanitizers: the threaded input-pipeline
core (worker pool + slot hand-off, csrc/data/loader_core.h) runs its multi-worker stress
test plain, under ASan+UBSan and under TSan.  GPU-side sanitizers are not available
on the MI355X pool; the RCCL communicator needs a GPU and is exercised by the GPU tests."""
import os
import subprocess

import pytest

from cloud_amd import _build


@pytest.mark.parametrize("sanitize", [None, "address", "thread"])
def test_loader_core_under_sanitizers(sanitize):
    exe = _build.build_loader_test(sanitize)
    env = dict(os.environ, ASAN_OPTIONS="verify_asan_link_order=0:detect_leaks=1",
               TSAN_OPTIONS="halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "loader_test: ok" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
