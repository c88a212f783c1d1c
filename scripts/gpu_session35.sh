#!/usr/bin/env bash
# Wide 128x256 tiles for memory-bound N=256 GEMMs: tests, microbench, bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "FAILED\|ERROR" gpurun_out/pytest_gpu.log && { echo "gpu tests failed"; exit 1; }
$S 300 smallk_wide.log python bench/smallk_gemm.py || exit 1
$S 300 bench_w1.log python bench.py --steps 20 --warmup 5 || exit 1
$S 300 bench_w0.log env CLOUD_AMD_GEMM_WIDE=0 python bench.py --steps 20 --warmup 5 || exit 1
$S 300 bench_w1b.log python bench.py --steps 20 --warmup 5 || exit 1
echo SESSION_DONE
