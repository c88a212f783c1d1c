#!/usr/bin/env bash
# BatchNorm apply passes: interleaved row groups (CLOUD_AMD_BN_APPLY_ILV) x grid size; end-to-end.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
for il in 0 1; do
  for b in 0 2048 8192; do
    CLOUD_AMD_BN_APPLY_ILV=$il CLOUD_AMD_BN_APPLY_BLOCKS=$b $S 200 r2s28_bw_${il}_$b.log python bench/bn_apply_bw.py || exit 1
  done
done
CLOUD_AMD_BN_APPLY_ILV=1 $S 600 r2s28_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
for i in 1 2; do
  CLOUD_AMD_BN_APPLY_ILV=0 $S 200 r2s28_bench_ilv0_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_BN_APPLY_ILV=1 $S 200 r2s28_bench_ilv1_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_BN_APPLY_ILV=1 CLOUD_AMD_BN_APPLY_BLOCKS=2048 $S 200 r2s28_bench_ilv1_2048_$i.log python bench.py --via-run 0 || exit 1
done
echo SESSION_DONE
