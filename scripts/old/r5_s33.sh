#!/usr/bin/env bash
# Round-5 session 33: long runs on the final tree (steady state): ResNet-50 200 steps, BERT 500.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s33}
$S 300 ${tag}_rn200.log python bench.py --steps 200 --warmup 10 || exit 1
$S 300 ${tag}_bert500.log python bench/bert_base_synth.py --steps 500 --warmup 10 || exit 1
for f in gpurun_out/${tag}_rn200.log gpurun_out/${tag}_bert500.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1) $(grep -o '"device_ms": {[^}]*}' $f | tail -1)"; done
echo SESSION_DONE
