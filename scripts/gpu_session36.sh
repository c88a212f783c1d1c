#!/usr/bin/env bash
# Epilogue: LDS reads batched per row group before the stores; wide-tile A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "FAILED\|ERROR" gpurun_out/pytest_gpu.log && { echo "gpu tests failed"; exit 1; }
$S 300 smallk_w1.log python bench/smallk_gemm.py || exit 1
$S 300 smallk_w0.log env CLOUD_AMD_GEMM_WIDE=0 python bench/smallk_gemm.py || exit 1
$S 300 bench_w1.log python bench.py --steps 20 --warmup 5 || exit 1
$S 300 bench_w0.log env CLOUD_AMD_GEMM_WIDE=0 python bench.py --steps 20 --warmup 5 || exit 1
echo SESSION_DONE
