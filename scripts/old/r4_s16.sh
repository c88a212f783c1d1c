#!/usr/bin/env bash
# Round-4 session 16: step-pacer depth A/B (2 / 3 / 4 / unbounded) on ResNet-50 and BERT.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s16}
for i in 1 2; do
for d in 2 3 4 0; do
CLOUD_AMD_MAX_STEPS_IN_FLIGHT=$d $S 240 ${tag}_rn_d${d}_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
done
done
for d in 2 3 0; do
CLOUD_AMD_MAX_STEPS_IN_FLIGHT=$d $S 240 ${tag}_bert_d${d}.log python bench/bert_base_synth.py || exit 1
done
for f in rn_d2_1 rn_d3_1 rn_d4_1 rn_d0_1 rn_d2_2 rn_d3_2 rn_d4_2 rn_d0_2 bert_d2 bert_d3 bert_d0; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log | tail -1)"; done
echo SESSION_DONE
