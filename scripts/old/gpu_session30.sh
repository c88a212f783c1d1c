#!/usr/bin/env bash
# Alternating A/B (BERT side-stream param grads), 3 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
for i in 1 2 3; do
  $S 200 bert_a0_$i.log env CLOUD_AMD_WGRAD_STREAM=0 python bench/bert_base_synth.py --steps 40 --warmup 8 || exit 1
  $S 200 bert_a1_$i.log python bench/bert_base_synth.py --steps 40 --warmup 8 || exit 1
done
echo SESSION_DONE
