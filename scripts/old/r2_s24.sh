#!/usr/bin/env bash
# Split-major XCD mapping of split-K grids (CLOUD_AMD_SPLIT_XCD): GPU tests, A/B, profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 600 r2s24_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/r2s24_pytest_gpu.log && ! grep -q " failed" gpurun_out/r2s24_pytest_gpu.log || { echo "GPU tests failed"; exit 1; }
for i in 1 2; do
  CLOUD_AMD_SPLIT_XCD=0 $S 200 r2s24_off_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_SPLIT_XCD=1 $S 200 r2s24_on_$i.log python bench.py --via-run 0 || exit 1
done
CLOUD_AMD_SPLIT_XCD=0 $S 200 r2s24_bert_off.log python bench/bert_base_synth.py --via-run 0 || exit 1
CLOUD_AMD_SPLIT_XCD=1 $S 200 r2s24_bert_on.log python bench/bert_base_synth.py --via-run 0 || exit 1
rm -f gpurun_out/r2s24_shapes.jsonl
CLOUD_AMD_WGRAD_STREAM=0 CLOUD_AMD_SHAPE_LOG=gpurun_out/r2s24_shapes.jsonl $S 300 r2s24_prof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/r2s24_prof -o run -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
echo SESSION_DONE
