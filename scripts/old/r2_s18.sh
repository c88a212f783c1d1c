#!/usr/bin/env bash
# Buffer-mode loaders (32-bit offsets, range-check zero fill): tests, A/B, BERT, roofline profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 200 r2s18_conv_test.log python -u -m pytest tests/test_kernels_gpu.py -v -k "conv or bottleneck or stem" --timeout 120 --timeout-method thread || exit 1
grep -q "FAILED\|ERROR" gpurun_out/r2s18_conv_test.log && { echo "conv tests failed"; exit 1; }
$S 500 r2s18_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
for i in 1 2; do
  CLOUD_AMD_TAPMASK=1 $S 200 r2s18_on_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_TAPMASK=0 $S 200 r2s18_off_$i.log python bench.py --via-run 0 || exit 1
done
rm -f gpurun_out/r2s18_shapes_rn.jsonl
CLOUD_AMD_WGRAD_STREAM=0 CLOUD_AMD_SHAPE_LOG=gpurun_out/r2s18_shapes_rn.jsonl $S 300 r2s18_prof_rn.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/r2s18_prof_rn -o run -- python bench.py --via-run 0 --steps 3 --warmup 2 || exit 1
$S 200 r2s18_bert.log python bench/bert_base_synth.py --via-run 0 || exit 1
echo SESSION_DONE
