#!/usr/bin/env bash
# Stem tail kernels with XCD-contiguous block ranges (reverted STEM_XCD switch in pool.hip): GPU tests, A/B, kernel times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 600 r2s34_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/r2s34_pytest_gpu.log && ! grep -q " failed" gpurun_out/r2s34_pytest_gpu.log || { echo "GPU tests failed"; exit 1; }
for i in 1 2 3; do
  STEM_XCD=0 $S 200 r2s34_bench_x0_$i.log python bench.py --via-run 0 || exit 1
  STEM_XCD=1 $S 200 r2s34_bench_x1_$i.log python bench.py --via-run 0 || exit 1
done
for x in 0 1; do
  STEM_XCD=$x CLOUD_AMD_WGRAD_STREAM=0 $S 300 r2s34_prof_x$x.log \
    rocprofv3 --kernel-trace --stats -d gpurun_out/r2s34_prof_x$x -o run -- python bench.py --via-run 0 --steps 3 --warmup 2 || exit 1
done
echo SESSION_DONE
