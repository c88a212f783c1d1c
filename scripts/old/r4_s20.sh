#!/usr/bin/env bash
# Round-4 session 20: 8-wave transform-A GEMMs (CLOUD_AMD_XA_WAVES=8: <= 128 registers, two
# 8-wave workgroups per CU) -- fold tests under it, then ResNet-50 A/B interleaved x3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s20}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
CLOUD_AMD_XA_WAVES=8 $S 300 ${tag}_fold_tests8.log python -u -m pytest tests/test_bn_fold_gpu.py -q --timeout 120 --timeout-method thread || exit 1
tail -3 gpurun_out/${tag}_fold_tests8.log
for i in 1 2 3; do
CLOUD_AMD_XA_WAVES=8 $S 240 ${tag}_w8_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 240 ${tag}_w4_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
done
rm -rf gpurun_out/${tag}_prof
CLOUD_AMD_XA_WAVES=8 CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_prof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof sgd_kernel > gpurun_out/${tag}_rn_step_kernels_w8.txt
rm -rf gpurun_out/${tag}_prof
head -12 gpurun_out/${tag}_rn_step_kernels_w8.txt
for f in w8_1 w4_1 w8_2 w4_2 w8_3 w4_3; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log | tail -1)"; done
echo SESSION_DONE
