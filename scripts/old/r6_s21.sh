#!/usr/bin/env bash
# Round-6 session 21: critical path on a high-priority stream (BERT, ResNet), in-process runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s21
for r in 1 2 3; do
$S 200 ${tag}_bert_base_$r.log python bench/bert_base_synth.py --via-run 0 --steps 30 --warmup 5 || exit 1
$S 200 ${tag}_bert_prio_$r.log python scripts/prio_probe.py bench/bert_base_synth.py --steps 30 --warmup 5 || exit 1
done
for r in 1 2; do
$S 200 ${tag}_rn_base_$r.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
$S 200 ${tag}_rn_prio_$r.log python scripts/prio_probe.py bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
