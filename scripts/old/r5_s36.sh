#!/usr/bin/env bash
# Round-5 session 36: BERT-base per-GPU batch sweep (64 = the bench default, 128, 256), two runs each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s36}
for r in 1 2; do
for b in 64 128 256; do
$S 200 ${tag}_b${b}_$r.log python bench/bert_base_synth.py --batch $b --steps 20 --warmup 5 || exit 1
echo "b${b}_$r $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_b${b}_$r.log | tail -1) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${tag}_b${b}_$r.log | tail -1) $(grep -o '"host_launch_rank0": {[^}]*}' gpurun_out/${tag}_b${b}_$r.log | tail -1)"
done
done
echo SESSION_DONE
