#!/usr/bin/env bash
# GELU / GELU' epilogue with the shared-exp erf: tests + alternating BERT runs vs previous numbers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "FAILED\|ERROR" gpurun_out/pytest_gpu.log && { echo "gpu tests failed"; exit 1; }
for i in 1 2 3; do
  $S 200 bert_gelu_$i.log python bench/bert_base_synth.py --steps 40 --warmup 8 || exit 1
done
$S 300 prof_bert.log env CLOUD_AMD_WGRAD_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert3 -o run -- python bench/bert_base_synth.py --steps 10 --warmup 3 || exit 1
echo SESSION_DONE
