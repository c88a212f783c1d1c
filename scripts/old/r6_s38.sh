#!/usr/bin/env bash
# Round-6 session 38: re-check the default-off one-pass input+weight gradient folds on the final
# tree (CLOUD_AMD_BN_FOLD_WGRAD1: stage-1 conv1; CLOUD_AMD_BN_FOLD_WGRAD2: stage-2 conv3), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s38
for r in 1 2 3; do
$S 200 ${tag}_rn_def_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD_WGRAD1=1 $S 200 ${tag}_rn_w1_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD_WGRAD2=1 $S 200 ${tag}_rn_w2_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
