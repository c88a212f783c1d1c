#!/usr/bin/env bash
# Round-4 session 30: fold tests incl. the deep fused-gradient cases; serialized step profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s30}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 300 ${tag}_fold.log python -u -m pytest tests/test_bn_fold_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_fold.log
rm -rf gpurun_out/${tag}_prof
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_prof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof sgd_kernel > gpurun_out/${tag}_rn_step_kernels.txt
rm -rf gpurun_out/${tag}_prof
tail -1 gpurun_out/${tag}_fold.log
head -12 gpurun_out/${tag}_rn_step_kernels.txt
echo SESSION_DONE
