#!/usr/bin/env bash
# Final-state verification: GPU tests, smoke, the driver's bench command (via run()), BERT, kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 600 r2s39_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/r2s39_pytest_gpu.log && ! grep -q " failed" gpurun_out/r2s39_pytest_gpu.log || { echo "GPU tests failed"; exit 1; }
$S 200 r2s39_smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S 300 r2s39_bench_driver.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 300 r2s39_bench_default.log python bench.py || exit 1
$S 300 r2s39_bert_via_run.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_SHARED_GPU=1 CLOUD_AMD_DIST_BACKEND=gloo CLOUD_AMD_NUM_GPUS=2 $S 300 r2s39_dp2_rehearsal.log python bench.py --gpus 2 --steps 4 --warmup 2 --batch 128 || exit 1
echo SESSION_DONE
