#!/usr/bin/env bash
# 128x256 / 8-wave tiles for wide forward 1x1 GEMMs with BN statistics (reverted WIDE_FWD switch, gemm.hip): tests, A/B, profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
WIDE_FWD=1 $S 600 r2s41_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/r2s41_pytest_gpu.log && ! grep -q " failed" gpurun_out/r2s41_pytest_gpu.log || { echo "GPU tests failed"; exit 1; }
for i in 1 2 3; do
  WIDE_FWD=0 $S 200 r2s41_bench_w0_$i.log python bench.py --via-run 0 || exit 1
  WIDE_FWD=1 $S 200 r2s41_bench_w1_$i.log python bench.py --via-run 0 || exit 1
done
rm -f gpurun_out/r2s41_shapes.jsonl
WIDE_FWD=1 CLOUD_AMD_WGRAD_STREAM=0 CLOUD_AMD_SHAPE_LOG=gpurun_out/r2s41_shapes.jsonl $S 300 r2s41_prof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/r2s41_prof -o run -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
echo SESSION_DONE
