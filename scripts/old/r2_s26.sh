#!/usr/bin/env bash
# Split-K workgroup target for the <= 128-channel weight gradients (CLOUD_AMD_WGRAD_BLOCKS_SMALLM), end-to-end.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
for i in 1 2; do
  for b in 512 1024 2048; do
    CLOUD_AMD_WGRAD_BLOCKS_SMALLM=$b $S 200 r2s26_sm${b}_$i.log python bench.py --via-run 0 || exit 1
  done
done
for b in 512 2048; do
  CLOUD_AMD_WGRAD_BLOCKS_SMALLM=$b CLOUD_AMD_WGRAD_STREAM=0 $S 200 r2s26_serial_sm${b}.log python bench.py --via-run 0 || exit 1
done
echo SESSION_DONE
