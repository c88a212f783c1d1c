#!/usr/bin/env bash
# BatchNorm apply-pass grid size (CLOUD_AMD_BN_APPLY_BLOCKS): bandwidth micro-benchmark, GPU tests, end-to-end.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
for b in 0 2048 4096 8192; do
  CLOUD_AMD_BN_APPLY_BLOCKS=$b $S 200 r2s27_bw_$b.log python bench/bn_apply_bw.py || exit 1
done
CLOUD_AMD_BN_APPLY_BLOCKS=4096 $S 600 r2s27_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
for i in 1 2; do
  for b in 0 2048 4096; do
    CLOUD_AMD_BN_APPLY_BLOCKS=$b $S 200 r2s27_bench_${b}_$i.log python bench.py --via-run 0 || exit 1
  done
done
echo SESSION_DONE
