#!/usr/bin/env bash
# Round-3 session 37: GPU clock / power / temperature sampled (rocm-smi, read-only, once a
# second) while the ResNet-50 bench repeats -- do the occasional 3x-slow runs coincide with
# a clock drop?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s37}
mkdir -p gpurun_out
( while true; do echo "T $(date +%T.%N | cut -c1-12)"; timeout 10 rocm-smi --showclocks --showpower --showtemp 2>/dev/null | grep -E "sclk|mclk|Power|Temperature" ; sleep 1; done ) > gpurun_out/${tag}_smi.log 2>&1 &
MON=$!
rc=0
for i in 1 2 3 4 5 6; do
echo "[run $i] $(date +%T.%N | cut -c1-12) start" >> gpurun_out/${tag}_smi.log
$S 240 ${tag}_rn_b512_${i}.log python bench.py --gpus 1 --steps 30 --warmup 5 --batch 512 || { rc=1; break; }
echo "[run $i] $(date +%T.%N | cut -c1-12) end" >> gpurun_out/${tag}_smi.log
done
kill $MON
for i in 1 2 3 4 5 6; do echo "run $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${tag}_rn_b512_$i.log | tail -1)"; done
grep -E "sclk|\[run" gpurun_out/${tag}_smi.log | head -80
echo SESSION_DONE
exit $rc
