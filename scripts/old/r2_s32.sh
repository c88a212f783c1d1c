#!/usr/bin/env bash
# Stem weight-gradient split-K target (CLOUD_AMD_STEM_WGRAD_BLOCKS) A/B; GPU tests; serialized profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 600 r2s32_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/r2s32_pytest_gpu.log && ! grep -q " failed" gpurun_out/r2s32_pytest_gpu.log || { echo "GPU tests failed"; exit 1; }
for i in 1 2 3; do
  CLOUD_AMD_STEM_WGRAD_BLOCKS=512 $S 200 r2s32_bench_stem512_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_STEM_WGRAD_BLOCKS=2048 $S 200 r2s32_bench_stem2048_$i.log python bench.py --via-run 0 || exit 1
done
rm -f gpurun_out/r2s32_shapes.jsonl
CLOUD_AMD_WGRAD_STREAM=0 CLOUD_AMD_SHAPE_LOG=gpurun_out/r2s32_shapes.jsonl $S 300 r2s32_prof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/r2s32_prof -o run -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
echo SESSION_DONE
