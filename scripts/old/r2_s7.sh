#!/usr/bin/env bash
# After the swizzled C-staging change: full GPU tests, bench x2, serialized profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 400 r2s7_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/r2s7_pytest_gpu.log && ! grep -q "FAILED\|ERROR" gpurun_out/r2s7_pytest_gpu.log || { echo "gpu tests failed"; exit 1; }
$S 200 r2s7_bench_1.log python bench.py || exit 1
$S 200 r2s7_bench_2.log python bench.py || exit 1
CLOUD_AMD_WGRAD_STREAM=0 $S 300 r2s7_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/r2s7_prof -o run -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
echo SESSION_DONE
