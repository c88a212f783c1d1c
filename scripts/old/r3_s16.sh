#!/usr/bin/env bash
# Round-3 session 16: batch sweep of the final ResNet-50 tree (b256 / b512 / b1024, twice each,
# interleaved), BERT weight-gradient split target A/B (512 vs 1024 workgroups).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s16}
for i in 1 2; do
for b in 256 512 1024; do
$S 240 ${tag}_rn_b${b}_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 --batch $b || exit 1
done
$S 240 ${tag}_bert_w1024_${i}.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_DENSE_WGRAD_BLOCKS=512 $S 240 ${tag}_bert_w512_${i}.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_DENSE_WGRAD_BLOCKS=2048 $S 240 ${tag}_bert_w2048_${i}.log python bench/bert_base_synth.py || exit 1
done
for f in rn_b256_1 rn_b512_1 rn_b1024_1 rn_b256_2 rn_b512_2 rn_b1024_2 bert_w1024_1 bert_w512_1 bert_w2048_1 bert_w1024_2 bert_w512_2 bert_w2048_2; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log)"; done
echo SESSION_DONE
