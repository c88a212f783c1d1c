#!/usr/bin/env bash
# 256 x 64 tall tiles for the <= 64-channel 3x3 convolutions (CLOUD_AMD_CONV_TALL): tests, shapes, end-to-end.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 600 r2s29_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/r2s29_pytest_gpu.log && ! grep -q " failed" gpurun_out/r2s29_pytest_gpu.log || { echo "GPU tests failed"; exit 1; }
CLOUD_AMD_CONV_TALL=0 $S 200 r2s29_shapes_tall0.log python bench/conv_shapes.py l1_c2 1024 || exit 1
CLOUD_AMD_CONV_TALL=1 $S 200 r2s29_shapes_tall1.log python bench/conv_shapes.py l1_c2 1024 || exit 1
for i in 1 2; do
  CLOUD_AMD_CONV_TALL=0 $S 200 r2s29_bench_tall0_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_CONV_TALL=1 $S 200 r2s29_bench_tall1_$i.log python bench.py --via-run 0 || exit 1
done
echo SESSION_DONE
