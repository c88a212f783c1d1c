#!/usr/bin/env bash
# Round-4 session 23: stage-1 projection-shortcut fusion (BN backward + dgrad + wgrad in one pass)
# -- fold tests, ResNet-50 A/B interleaved x3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s23}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 300 ${tag}_fold_tests.log python -u -m pytest tests/test_bn_fold_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_fold_tests.log
for i in 1 2 3; do
$S 240 ${tag}_ds_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD_WGRAD_DS=0 $S 240 ${tag}_nods_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
done
for f in ds_1 nods_1 ds_2 nods_2 ds_3 nods_3; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log | tail -1)"; done
echo SESSION_DONE
