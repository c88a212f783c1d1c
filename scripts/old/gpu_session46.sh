#!/usr/bin/env bash
# Identity-block residual gradient gated in conv1's dgrad epilogue (no dres write): tests, bench x2, profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "FAILED\|ERROR" gpurun_out/pytest_gpu.log && { echo "gpu tests failed"; exit 1; }
$S 300 bench_a.log python bench.py --steps 20 --warmup 5 || exit 1
$S 300 bench_b.log python bench.py --steps 20 --warmup 5 || exit 1
$S 400 prof.log env CLOUD_AMD_WGRAD_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ser9 -o run -- python bench.py --steps 6 --warmup 2 || exit 1
echo SESSION_DONE
