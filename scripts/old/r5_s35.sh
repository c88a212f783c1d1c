#!/usr/bin/env bash
# Round-5 session 35: BERT bench with the host-launch timing fields (is the step host-bound?).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s35}
for r in 1 2; do
$S 200 ${tag}_bert_$r.log python bench/bert_base_synth.py --steps 30 --warmup 5 || exit 1
echo "bert_$r $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_bert_$r.log | tail -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${tag}_bert_$r.log | tail -1) $(grep -o '"host_launch_rank0": {[^}]*}' gpurun_out/${tag}_bert_$r.log | tail -1)"
done
echo SESSION_DONE
