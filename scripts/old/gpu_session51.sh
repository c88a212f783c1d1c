#!/usr/bin/env bash
# Verification after the CLOUD_AMD_DEBUG_SYNC launch check: GPU tests (normal and with every
# native launch synchronised), smoke, headline bench (must be unchanged by the check).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
grep -q "FAILED\|ERROR" gpurun_out/pytest_gpu.log && { echo "gpu tests failed"; exit 1; }
$S 300 pytest_dbg.log env CLOUD_AMD_DEBUG_SYNC=1 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "FAILED\|ERROR" gpurun_out/pytest_dbg.log && { echo "debug-sync gpu tests failed"; exit 1; }
$S 300 smoke.log python __graft_entry__.py smoke || exit 1
for i in 1 2; do $S 300 bench_$i.log python bench.py || exit 1; done
echo SESSION_DONE
