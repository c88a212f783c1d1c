#!/usr/bin/env bash
# Round-4 session 22: 8-wave 128 x 64 transform-A GEMMs (stage 1, CLOUD_AMD_XA_WAVES_N64=1) --
# fold tests under it, ResNet-50 A/B interleaved x3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s22}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
CLOUD_AMD_XA_WAVES_N64=1 $S 300 ${tag}_fold_tests.log python -u -m pytest tests/test_bn_fold_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_fold_tests.log
for i in 1 2 3; do
CLOUD_AMD_XA_WAVES_N64=1 $S 240 ${tag}_n64w8_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 240 ${tag}_def_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
done
for f in n64w8_1 def_1 n64w8_2 def_2 n64w8_3 def_3; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log | tail -1)"; done
echo SESSION_DONE
