#!/usr/bin/env bash
# Round-6 session 43: the 8-wave 128 x 256 transform-A form moved behind the experimental build --
# fold / kernel GPU tests, one ResNet-50 run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s43
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 600 ${tag}_kt.log python -u -m pytest tests/test_bn_fold_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread || exit 1
chk ${tag}_kt.log
tail -1 gpurun_out/${tag}_kt.log
$S 200 ${tag}_rn.log python bench.py --steps 20 --warmup 5 || exit 1
echo "$(grep -o '"value": [0-9.]*' gpurun_out/${tag}_rn.log | tail -1)"
echo SESSION_DONE
