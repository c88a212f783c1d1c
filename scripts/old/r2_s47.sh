#!/usr/bin/env bash
# BERT dense weight-gradient split target 1024 (default) vs 2048.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
for i in 1 2 3; do
  $S 200 r2s47_bert_1024_$i.log python bench/bert_base_synth.py --via-run 0 || exit 1
  CLOUD_AMD_DENSE_WGRAD_BLOCKS=2048 $S 200 r2s47_bert_2048_$i.log python bench/bert_base_synth.py --via-run 0 || exit 1
done
echo SESSION_DONE
