#!/usr/bin/env bash
# pp256 core correctness test + full GPU suite after the GEMM-core changes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 200 r2s13_pp256_test.log python -u -m pytest tests/test_gemm_pp256_gpu.py -v --timeout 120 --timeout-method thread || exit 1
grep -q "FAILED\|ERROR" gpurun_out/r2s13_pp256_test.log && { echo "pp256 test failed"; exit 1; }
$S 400 r2s13_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
echo SESSION_DONE
