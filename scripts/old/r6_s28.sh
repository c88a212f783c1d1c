#!/usr/bin/env bash
# Round-6 session 28: serialized ResNet-50 step profiles, default fold sites vs every stage folded
# on the 128 x 256 transform-A tiles (CLOUD_AMD_BN_FOLD_MAX_N=512).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s28
for v in 128 512; do
rm -rf gpurun_out/${tag}_rprof
CLOUD_AMD_BN_FOLD_MAX_N=$v CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_rprof_$v.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_rprof -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_rprof sgd_kernel > gpurun_out/${tag}_rn_step_kernels_$v.txt || true
rm -rf gpurun_out/${tag}_rprof
head -3 gpurun_out/${tag}_rn_step_kernels_$v.txt
done
echo SESSION_DONE
