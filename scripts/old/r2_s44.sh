#!/usr/bin/env bash
# Final tree: GPU tests (with the free-port multi-process tests), smoke, the driver's bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 600 r2s44_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/r2s44_pytest_gpu.log && ! grep -q " failed" gpurun_out/r2s44_pytest_gpu.log || { echo "GPU tests failed"; exit 1; }
$S 200 r2s44_smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S 300 r2s44_bench_driver.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
echo SESSION_DONE
