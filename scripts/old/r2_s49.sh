#!/usr/bin/env bash
# Flattened-halo conv with 64-wide N tiles at every width: subprocess GPU test, shapes, A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 400 r2s49_halo_test.log python -u -m pytest tests/test_conv_halo_gpu.py -x -q --timeout 300 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/r2s49_halo_test.log && ! grep -q " failed" gpurun_out/r2s49_halo_test.log || { echo "halo test failed"; exit 1; }
for t in l1_c2 l2_c2 l3_c2 l4_c2; do
  CLOUD_AMD_CONV_HALO=1 $S 200 r2s49_shape_${t}_h1.log python bench/conv_shapes.py $t 1024 || exit 1
  CLOUD_AMD_CONV_HALO=0 $S 200 r2s49_shape_${t}_h0.log python bench/conv_shapes.py $t 1024 || exit 1
done
for i in 1 2; do
  CLOUD_AMD_CONV_HALO=0 $S 200 r2s49_bench_h0_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_CONV_HALO=1 $S 200 r2s49_bench_h1_$i.log python bench.py --via-run 0 || exit 1
done
echo SESSION_DONE
