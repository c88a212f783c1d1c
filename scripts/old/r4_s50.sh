#!/usr/bin/env bash
# Round-4 session 50: long-run stability of the final tree (100 timed steps, step statistics).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s50}
for r in 1 2; do
$S 300 ${tag}_rn100_${r}.log python bench.py --gpus 1 --steps 100 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1) $(grep -o '"max_over_median": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
