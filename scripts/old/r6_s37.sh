#!/usr/bin/env bash
# Round-6 session 37: stock PyTorch-ROCm comparators next to the final tree, same box --
# ResNet-50 (torch.nn + AMP, MIOpen find off) and BERT-base (HF transformers + autocast +
# fused AdamW), then the framework's benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s37
$S 500 ${tag}_stock_rn.log python bench/stock_resnet50.py --steps 20 --warmup 5 || exit 1
$S 300 ${tag}_stock_bert.log python bench/bert_base_synth.py --stock 1 --steps 20 --warmup 5 || exit 1
$S 200 ${tag}_rn.log python bench.py --steps 20 --warmup 5 || exit 1
$S 200 ${tag}_bert.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
for f in gpurun_out/${tag}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
