#!/usr/bin/env bash
# Round-6 session 41: register-staged fragments with the next tile's DMA before this tile's MFMAs
# for the implicit-GEMM convolutions (CLOUD_AMD_CONV_RP) -- conv tests with it on, stage 2-4 3x3
# shapes on / off, ResNet-50 A/B interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s41
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
CLOUD_AMD_CONV_RP=1 $S 400 ${tag}_kt.log python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv or dgrad or fused_bottleneck" || exit 1
chk ${tag}_kt.log
tail -1 gpurun_out/${tag}_kt.log
for sh in l2_c2 l3_c2 l4_c2 l2_c2_s2; do
$S 120 ${tag}_cs0_$sh.log python bench/conv_shapes.py $sh 1024 || exit 1
CLOUD_AMD_CONV_RP=1 $S 120 ${tag}_cs1_$sh.log python bench/conv_shapes.py $sh 1024 || exit 1
echo "$sh off $(grep -o '{.*}' gpurun_out/${tag}_cs0_$sh.log | tail -1)"
echo "$sh on  $(grep -o '{.*}' gpurun_out/${tag}_cs1_$sh.log | tail -1)"
done
for r in 1 2; do
$S 200 ${tag}_rn_off_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_CONV_RP=1 $S 200 ${tag}_rn_on_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
