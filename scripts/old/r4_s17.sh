#!/usr/bin/env bash
# Round-4 session 17: stage-1 fused input+weight gradient (with cross-tile prefetch) on vs off,
# interleaved; serialized step profile of the default tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s17}
for i in 1 2 3; do
$S 240 ${tag}_dw_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD_WGRAD=0 $S 240 ${tag}_nodw_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
done
rm -rf gpurun_out/${tag}_prof
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_prof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof sgd_kernel > gpurun_out/${tag}_rn_step_kernels.txt
rm -rf gpurun_out/${tag}_prof
head -12 gpurun_out/${tag}_rn_step_kernels.txt
for f in dw_1 nodw_1 dw_2 nodw_2 dw_3 nodw_3; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log | tail -1)"; done
echo SESSION_DONE
