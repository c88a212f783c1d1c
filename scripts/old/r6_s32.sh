#!/usr/bin/env bash
# Round-6 session 32: confirmation A/B of the stage-3 BN folds on two-deep 128 x 256 tiles
# (CLOUD_AMD_BN_FOLD_MAX_N=256 CLOUD_AMD_XA_N256=3) against the default, three interleaved pairs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s32
for r in 1 2 3; do
$S 200 ${tag}_rn_def_$r.log python bench.py --steps 30 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD_MAX_N=256 CLOUD_AMD_XA_N256=3 $S 200 ${tag}_rn_n256d_$r.log python bench.py --steps 30 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
