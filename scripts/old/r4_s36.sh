#!/usr/bin/env bash
# Round-4 session 36: BERT dense weight-gradient split target around 768.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s36}
for r in 1 2; do
for b in 1024 768 512 640; do
CLOUD_AMD_DENSE_WGRAD_BLOCKS=$b $S 240 ${tag}_bert_wb${b}_${r}.log python bench/bert_base_synth.py || exit 1
done
done
for f in gpurun_out/${tag}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
