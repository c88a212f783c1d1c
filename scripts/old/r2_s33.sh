#!/usr/bin/env bash
# BN statistics first-level reduce: up to 512 groups (CLOUD_AMD_BN_GROUPS_MAX) vs the old 64; GPU tests; A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 600 r2s33_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/r2s33_pytest_gpu.log && ! grep -q " failed" gpurun_out/r2s33_pytest_gpu.log || { echo "GPU tests failed"; exit 1; }
for i in 1 2 3; do
  CLOUD_AMD_BN_GROUPS_MAX=64 $S 200 r2s33_bench_g64_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_BN_GROUPS_MAX=512 $S 200 r2s33_bench_g512_$i.log python bench.py --via-run 0 || exit 1
done
CLOUD_AMD_WGRAD_STREAM=0 $S 300 r2s33_prof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/r2s33_prof -o run -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
echo SESSION_DONE
