#!/usr/bin/env bash
# Round-4 session 24: serialized ResNet-50 b1024 step profile of the current default tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s24}
rm -rf gpurun_out/${tag}_prof
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_prof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof sgd_kernel > gpurun_out/${tag}_rn_step_kernels.txt
rm -rf gpurun_out/${tag}_prof
head -40 gpurun_out/${tag}_rn_step_kernels.txt
echo SESSION_DONE
