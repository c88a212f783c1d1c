#!/usr/bin/env bash
# Round-4 session 12: fused conv3 input+weight gradient (stage 1) -- numerics vs fp32, model-level
# closeness, then ResNet-50 A/B (CLOUD_AMD_BN_FOLD_WGRAD=1 default vs 0), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s12}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 300 ${tag}_fold_tests.log python -u -m pytest tests/test_bn_fold_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_fold_tests.log
for i in 1 2; do
$S 240 ${tag}_dw_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD_WGRAD=0 $S 240 ${tag}_nodw_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
done
for f in dw_1 nodw_1 dw_2 nodw_2; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log | tail -1)"; done
echo SESSION_DONE
