#!/usr/bin/env bash
# Two-pass (64-row) epilogue staging: LDS per 128x128 block 34.8 -> 32 KB (5 blocks/CU).
# Full GPU suite, serialized kernel profile, headline bench x3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
grep -q "FAILED\|ERROR" gpurun_out/pytest_gpu.log && { echo "gpu tests failed"; exit 1; }
$S 300 prof.log env CLOUD_AMD_WGRAD_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 6 --warmup 2 || exit 1
for i in 1 2 3; do $S 200 bench_$i.log python bench.py || exit 1; done
$S 200 smallk.log python bench/smallk_gemm.py || exit 1
echo SESSION_DONE
