#!/usr/bin/env bash
# Round-4 session 5: stock PyTorch-ROCm comparators at the headline configs, same box as
# cloud_amd: ResNet-50 b1024 (channels_last + AMP + MIOpen, torch.optim SGD foreach), HF BERT b64.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s5}
$S 240 ${tag}_rn.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 600 ${tag}_stock_rn.log python bench/stock_resnet50.py --batch 1024 --steps 20 --warmup 5 || exit 1
$S 240 ${tag}_bert.log python bench/bert_base_synth.py || exit 1
$S 400 ${tag}_stock_bert.log python bench/bert_base_synth.py --stock 1 --steps 20 --warmup 5 || exit 1
for f in rn stock_rn bert stock_bert; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log | tail -1)"; done
echo SESSION_DONE
