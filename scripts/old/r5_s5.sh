#!/usr/bin/env bash
# Round-5 session 5: honest stock row -- stock PyTorch ResNet-50 b1024 with MIOpen find
# (torch.backends.cudnn.benchmark = True), same box and session as cloud_amd via run().
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s5}
$S 200 ${tag}_rn.log python bench.py --steps 20 --warmup 5 || exit 1
$S 1050 ${tag}_stock_bm1.log python bench/stock_resnet50.py --benchmark 1 --steps 20 --warmup 5 || exit 1
for f in gpurun_out/${tag}_rn.log gpurun_out/${tag}_stock_bm1.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1) $(grep -o '"first_step_latency_s": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
