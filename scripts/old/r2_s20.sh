#!/usr/bin/env bash
# Knob sweep on the current kernels: weight-gradient split target, pp256 core for the plain/partial GEMMs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
for i in 1 2; do
  $S 200 r2s20_base_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_WGRAD_BLOCKS=2048 $S 200 r2s20_wb2048_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_WGRAD_BLOCKS=512 $S 200 r2s20_wb512_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_GEMM_CORE=pp256 $S 200 r2s20_pp256_$i.log python bench.py --via-run 0 || exit 1
done
echo SESSION_DONE
