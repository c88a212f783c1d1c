#!/usr/bin/env bash
# Round-6 session 48: projection-shortcut BN backward folded into the sparse strided shortcut
# input-gradient GEMM (CLOUD_AMD_BN_FOLD_DS) -- kernel + block tests with it on, ResNet-50 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s48
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
CLOUD_AMD_BN_FOLD_DS=1 $S 600 ${tag}_kt.log python -u -m pytest tests/test_kernels_gpu.py tests/test_bn_fold_gpu.py -x -q --timeout 200 --timeout-method thread -k "strided_shortcut or sparse or fused_bottleneck or resnet" || exit 1
chk ${tag}_kt.log
tail -1 gpurun_out/${tag}_kt.log
for r in 1 2 3; do
$S 200 ${tag}_rn_off_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD_DS=1 $S 200 ${tag}_rn_on_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
