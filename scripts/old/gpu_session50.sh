#!/usr/bin/env bash
# LayerNorm backward with up to 1024 blocks (2 rows per wave at BERT's 8192 rows).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 pytest_t.log python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "FAILED\|ERROR" gpurun_out/pytest_t.log && { echo "gpu tests failed"; exit 1; }
$S 300 prof_bert.log env CLOUD_AMD_WGRAD_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert4 -o run -- python bench/bert_base_synth.py --steps 10 --warmup 3 || exit 1
for i in 1 2; do $S 200 bert_$i.log python bench/bert_base_synth.py --steps 40 --warmup 8 || exit 1; done
echo SESSION_DONE
