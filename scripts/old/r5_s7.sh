#!/usr/bin/env bash
# Round-5 session 7: LDS-resident 3x3 convolution (ca_conv_halo.h) numerics, then the conv and
# BN-fold GPU tests, ResNet-50 A/B with the halo kernel off / on, a serialized step profile,
# 128 x 192 tiles on BERT forward shapes, and the stock row with MIOpen find.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s7}
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$S 240 ${tag}_halo.log $PT tests/test_conv_halo_gpu.py || exit 1
grep -q " passed" gpurun_out/${tag}_halo.log && ! grep -q "FAILED\|Error" gpurun_out/${tag}_halo.log || { echo HALO_FAILED; exit 1; }
$S 600 ${tag}_conv.log $PT tests/test_bn_fold_gpu.py tests/test_kernels_gpu.py tests/test_no_library_fallback_gpu.py || exit 1
CLOUD_AMD_CONV_HALO=0 $S 200 ${tag}_rn_h0.log python bench.py --steps 20 --warmup 5 || exit 1
$S 200 ${tag}_rn_h1.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_CONV_HALO=0 $S 200 ${tag}_rn_h0b.log python bench.py --steps 20 --warmup 5 || exit 1
$S 200 ${tag}_rn_h1b.log python bench.py --steps 20 --warmup 5 || exit 1
for f in gpurun_out/${tag}_rn_h*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_rprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_rprof -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_rprof sgd_kernel > gpurun_out/${tag}_rn_step_kernels.txt 2>&1 || true
head -30 gpurun_out/${tag}_rn_step_kernels.txt 2>/dev/null
GB_VARIANTS=glds128,g128x192,p8h2 $S 200 ${tag}_gb.log bin/gemm_bench 20 8192,2304,768,0 8192,3072,768,0 8192,768,3072,0 8192,768,768,0 4096,4096,4096,0 || exit 1
grep -h '"variant"' gpurun_out/${tag}_gb.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('%-9s %5d %5d %5d L%d %8.1f us %7.1f TF bad=%d rel=%.2e' % (d['variant'],d['M'],d['N'],d['K'],d['layout'],d['us'],d['TF'],d['bad'],d['rel_l2']))"
$S 900 ${tag}_stock_bm1.log python bench/stock_resnet50.py --benchmark 1 --steps 20 --warmup 5 || exit 1
echo "$(grep -o '"value": [0-9.]*' gpurun_out/${tag}_stock_bm1.log | tail -1) $(grep -o '"first_step_latency_s": [0-9.]*' gpurun_out/${tag}_stock_bm1.log | tail -1)"
echo SESSION_DONE
