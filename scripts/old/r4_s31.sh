#!/usr/bin/env bash
# Round-4 session 31: which stages the bn3 fold pays at (CLOUD_AMD_BN_FOLD_MAX_N: 4096 = every
# stage, 256 = stages 1-3, 128 = stages 1-2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s31}
for r in 1 2; do
for n in 4096 256 128; do
CLOUD_AMD_BN_FOLD_MAX_N=$n $S 240 ${tag}_rn_n${n}_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
done
done
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
