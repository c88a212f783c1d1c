#!/usr/bin/env bash
# BERT kernel profile + ResNet batch-size probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 prof_bert.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o run -- python bench/bert_base_synth.py --steps 10 --warmup 3 || exit 1
$S 300 bench_b512.log python bench.py --steps 20 --warmup 5 --batch 512 || exit 1
$S 300 bench_b128.log python bench.py --steps 20 --warmup 5 --batch 128 || exit 1
echo SESSION_DONE
