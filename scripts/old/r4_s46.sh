#!/usr/bin/env bash
# Round-4 session 46: stem weight-gradient split target on the final tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s46}
for r in 1 2; do
$S 240 ${tag}_rn_default_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_STEM_WGRAD_BLOCKS=1024 $S 240 ${tag}_rn_sw1024_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_STEM_WGRAD_BLOCKS=4096 $S 240 ${tag}_rn_sw4096_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
