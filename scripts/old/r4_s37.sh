#!/usr/bin/env bash
# Round-4 session 37: BERT run-ahead depth and side-stream weight gradients.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s37}
for r in 1 2; do
$S 240 ${tag}_bert_default_${r}.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_MAX_STEPS_IN_FLIGHT=3 $S 240 ${tag}_bert_d3_${r}.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_MAX_STEPS_IN_FLIGHT=4 $S 240 ${tag}_bert_d4_${r}.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_ATTN_FUSED_BWD=0 $S 240 ${tag}_bert_attn0_${r}.log python bench/bert_base_synth.py || exit 1
done
for f in gpurun_out/${tag}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
