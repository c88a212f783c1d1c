#!/usr/bin/env bash
# Weight-gradient split target below 512; combined with the pp256 core.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
for i in 1 2; do
  CLOUD_AMD_WGRAD_BLOCKS=512 $S 200 r2s21_wb512_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_WGRAD_BLOCKS=256 $S 200 r2s21_wb256_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_WGRAD_BLOCKS=384 $S 200 r2s21_wb384_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_WGRAD_BLOCKS=512 CLOUD_AMD_GEMM_CORE=pp256 $S 200 r2s21_wb512pp_$i.log python bench.py --via-run 0 || exit 1
done
echo SESSION_DONE
