#!/usr/bin/env bash
# Round-5 session 10: halo dgrad statistics epilogue with up-front loads and the vectorized
# rotated-filter build; numerics, ResNet-50 A/B (halo off / on), serialized step profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s10}
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$S 300 ${tag}_t.log $PT tests/test_conv_halo_gpu.py tests/test_bn_finalize_gpu.py tests/test_bn_fold_gpu.py tests/test_gemm_256x96_gpu.py tests/test_gemm_streamk_gpu.py || exit 1
grep -q "FAILED\|Error" gpurun_out/${tag}_t.log && { echo T_FAILED; tail -30 gpurun_out/${tag}_t.log; exit 1; }
grep -E "passed|failed" gpurun_out/${tag}_t.log
GB_VARIANTS=glds128,g128x96,g256x96 $S 120 ${tag}_gb.log bin/gemm_bench 10 8192,2304,768,0 8192,768,3072,0 || exit 1
grep -h '"variant"' gpurun_out/${tag}_gb.log | cut -c1-160
$S 120 ${tag}_cs.log python bench/conv_shapes.py l1_c2 1024 || exit 1
grep tag gpurun_out/${tag}_cs.log
for r in 1 2; do
$S 200 ${tag}_rn_h1_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_CONV_HALO=0 $S 200 ${tag}_rn_h0_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_rprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_rprof -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_rprof sgd_kernel > gpurun_out/${tag}_rn_step_kernels.txt 2>&1 || true
head -16 gpurun_out/${tag}_rn_step_kernels.txt
grep halo gpurun_out/${tag}_rn_step_kernels.txt | head -8
for r in 1 2; do
$S 200 ${tag}_bert_q1_$r.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_GEMM_256X96=0 $S 200 ${tag}_bert_q0_$r.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_bert_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
