#!/usr/bin/env bash
# Stem-tail fusion: new test, full GPU tests, same-box A/B of the bench (tail on/off), profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 200 r2s10_stem_test.log python -u -m pytest tests/test_stem_tail_gpu.py -v --timeout 120 --timeout-method thread || exit 1
grep -q "FAILED\|ERROR" gpurun_out/r2s10_stem_test.log && { echo "stem test failed"; exit 1; }
$S 400 r2s10_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "FAILED\|ERROR" gpurun_out/r2s10_pytest_gpu.log && { echo "gpu tests failed"; exit 1; }
for i in 1 2; do
  CLOUD_AMD_STEM_TAIL=1 $S 200 r2s10_on_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_STEM_TAIL=0 $S 200 r2s10_off_$i.log python bench.py --via-run 0 || exit 1
done
CLOUD_AMD_WGRAD_STREAM=0 $S 300 r2s10_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/r2s10_prof -o run -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
for b in 64 128 256; do
  $S 200 r2s10_bert_b$b.log python bench/bert_base_synth.py --via-run 0 --batch $b || exit 1
done
echo SESSION_DONE
