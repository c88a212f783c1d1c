#!/usr/bin/env bash
# Round-4 session 35: knob sweep on the current tree -- ResNet-50 BN apply grid and side-stream
# weight gradients; BERT dense weight-gradient split target.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s35}
for r in 1 2; do
$S 240 ${tag}_rn_default_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_APPLY_BLOCKS=2048 $S 240 ${tag}_rn_ab2048_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_APPLY_BLOCKS=1024 $S 240 ${tag}_rn_ab1024_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
done
for r in 1 2; do
$S 240 ${tag}_bert_default_${r}.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_DENSE_WGRAD_BLOCKS=2048 $S 240 ${tag}_bert_wb2048_${r}.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_DENSE_WGRAD_BLOCKS=768 $S 240 ${tag}_bert_wb768_${r}.log python bench/bert_base_synth.py || exit 1
done
for f in gpurun_out/${tag}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
