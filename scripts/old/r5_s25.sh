#!/usr/bin/env bash
# Round-5 session 25: the stem-tail pooling kernels rewritten for VALU (integer-key max,
# branch-free backward gather): pooling / stem / ResNet GPU tests, the kernel microbench,
# and two ResNet-50 bench runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s25}
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
$S 400 ${tag}_tests.log $PYT tests/test_stem_tail_gpu.py tests/test_kernels_gpu.py tests/test_bn_fold_gpu.py tests/test_no_library_fallback_gpu.py || exit 1
grep -q " passed" gpurun_out/${tag}_tests.log && ! grep -q "failed" gpurun_out/${tag}_tests.log || { echo "tests failed"; exit 1; }
$S 120 ${tag}_micro.log python bench/stem_tail.py || exit 1
for r in 1 2; do
  $S 200 ${tag}_rn_$r.log python bench.py --steps 20 --warmup 5 || exit 1
  echo "rn_$r $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_rn_$r.log | tail -1)"
done
echo SESSION_DONE
