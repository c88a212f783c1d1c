#!/usr/bin/env bash
# Round-6 session 36: long runs on the final tree (ResNet-50 200 steps, BERT 500 steps): slow
# steps, allocator segments requested after warmup (BERT now queues three steps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s36
$S 400 ${tag}_rn_long.log python bench.py --steps 200 --warmup 5 || exit 1
$S 400 ${tag}_bert_long.log python bench/bert_base_synth.py --steps 500 --warmup 6 || exit 1
for f in gpurun_out/${tag}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1) $(grep -o '"max_steps_in_flight": [0-9]*' $f | tail -1)"; done
echo SESSION_DONE
