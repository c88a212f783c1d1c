#!/usr/bin/env bash
# Round-4 session 32: fold knobs around the new default (stages 1-2): stage 1 only; no forward fold.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s32}
for r in 1 2; do
$S 240 ${tag}_rn_default_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD_MAX_N=64 $S 240 ${tag}_rn_n64_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD_FWD=0 $S 240 ${tag}_rn_nofwd_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
