#!/usr/bin/env bash
# Lagged side-stream joins (reverted SIDE_LAG switch: runtime/side_stream.py lagged joins): GPU tests, ResNet-50 and BERT A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 600 r2s31_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/r2s31_pytest_gpu.log && ! grep -q " failed" gpurun_out/r2s31_pytest_gpu.log || { echo "GPU tests failed"; exit 1; }
for i in 1 2; do
  for l in 0 1 2; do
    SIDE_LAG=$l $S 200 r2s31_bench_lag${l}_$i.log python bench.py --via-run 0 || exit 1
  done
done
for l in 0 1 2; do
  SIDE_LAG=$l $S 200 r2s31_bert_lag${l}.log python bench/bert_base_synth.py --via-run 0 || exit 1
done
echo SESSION_DONE
