#!/usr/bin/env bash
# Round-4 session 51: stock PyTorch-ROCm ResNet-50 vs the final tree, same box, same session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s51}
$S 240 ${tag}_rn.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 900 ${tag}_stock.log python bench/stock_resnet50.py || exit 1
for f in gpurun_out/${tag}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
