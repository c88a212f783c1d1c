#!/usr/bin/env bash
# Flattened-halo 3x3 stride-1 forward convolution (CLOUD_AMD_CONV_HALO): GPU tests with it on, shapes, A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
CLOUD_AMD_CONV_HALO=1 $S 600 r2s48_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/r2s48_pytest_gpu.log && ! grep -q " failed" gpurun_out/r2s48_pytest_gpu.log || { echo "GPU tests failed"; exit 1; }
for h in 0 1; do
  for t in l1_c2 l2_c2 l3_c2 l4_c2; do
    CLOUD_AMD_CONV_HALO=$h $S 200 r2s48_shape_${t}_h$h.log python bench/conv_shapes.py $t 1024 || exit 1
  done
done
for i in 1 2; do
  CLOUD_AMD_CONV_HALO=0 $S 200 r2s48_bench_h0_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_CONV_HALO=1 $S 200 r2s48_bench_h1_$i.log python bench.py --via-run 0 || exit 1
done
echo SESSION_DONE
