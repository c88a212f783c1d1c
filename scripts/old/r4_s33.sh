#!/usr/bin/env bash
# Round-4 session 33: split-K workgroup targets of the convolution weight gradients.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s33}
for r in 1 2; do
$S 240 ${tag}_rn_default_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_WGRAD_BLOCKS=1024 $S 240 ${tag}_rn_wb1024_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_WGRAD_BLOCKS=256 $S 240 ${tag}_rn_wb256_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_WGRAD_BLOCKS_SMALLM=1024 $S 240 ${tag}_rn_sm1024_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
