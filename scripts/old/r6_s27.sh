#!/usr/bin/env bash
# Round-6 session 27: 128 x 256 transform-A tiles (BN folded into the 1x1 GEMMs at N = 256 / 512)
# -- fold tests, ResNet-50 A/B over CLOUD_AMD_BN_FOLD_MAX_N (128 = stages 1-2 only, 512 = every
# stage) and CLOUD_AMD_XA_N256 (1 = 16-wave, 2 = 8-wave), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s27
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 600 ${tag}_kt.log python -u -m pytest tests/test_bn_fold_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "fold or bnbwd or bnapply or fused_bottleneck" || exit 1
chk ${tag}_kt.log
tail -2 gpurun_out/${tag}_kt.log
for r in 1 2; do
CLOUD_AMD_BN_FOLD_MAX_N=128 $S 200 ${tag}_rn_n128_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD_MAX_N=512 $S 200 ${tag}_rn_n512w16_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD_MAX_N=512 CLOUD_AMD_XA_N256=2 $S 200 ${tag}_rn_n512w8_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD_MAX_N=256 $S 200 ${tag}_rn_n256w16_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
