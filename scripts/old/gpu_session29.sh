#!/usr/bin/env bash
# BERT: weight/bias gradients on the side stream (A/B); regression tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "FAILED\|ERROR" gpurun_out/pytest_gpu.log && { echo "gpu tests failed"; exit 1; }
$S 300 bert_ws1.log python bench/bert_base_synth.py --steps 30 --warmup 5 || exit 1
$S 300 bert_ws0.log env CLOUD_AMD_WGRAD_STREAM=0 python bench/bert_base_synth.py --steps 30 --warmup 5 || exit 1
$S 300 bert_ws1b.log python bench/bert_base_synth.py --steps 30 --warmup 5 || exit 1
$S 300 bench.log python bench.py --steps 20 --warmup 5 || exit 1
echo SESSION_DONE
