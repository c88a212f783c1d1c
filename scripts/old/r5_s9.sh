#!/usr/bin/env bash
# Round-5 session 9: halo conv with the chunk-major patch + DPP statistics, one-launch BN
# finalize with 1024-thread groups: numerics, shape timing, counters, ResNet-50 A/B runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s9}
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$S 200 ${tag}_t.log $PT tests/test_bn_finalize_gpu.py tests/test_conv_halo_gpu.py || exit 1
grep -q "FAILED\|Error" gpurun_out/${tag}_t.log && { echo T_FAILED; tail -30 gpurun_out/${tag}_t.log; exit 1; }
$S 120 ${tag}_cs.log python bench/conv_shapes.py l1_c2 1024 || exit 1
grep tag gpurun_out/${tag}_cs.log
out=gpurun_out/${tag}_pmc; mkdir -p $out
C="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
$S 90 ${tag}_pmc1.log timeout -s KILL 80 rocprofv3 --kernel-trace --pmc $C -d $out/p1 -o p1 --output-format csv -- python bench/conv_shapes.py l1_c2 1024 || exit 1
python3 scripts/pmc_clock.py $out > gpurun_out/${tag}_pmc_clock.txt 2>&1 || true
grep -i "halo" gpurun_out/${tag}_pmc_clock.txt | head -6
for r in 1 2; do
CLOUD_AMD_BN_FIN_MERGED=0 $S 200 ${tag}_rn_f0_$r.log python bench.py --steps 20 --warmup 5 || exit 1
$S 200 ${tag}_rn_f1_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_CONV_HALO=0 $S 200 ${tag}_rn_h0_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_rprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_rprof -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_rprof sgd_kernel > gpurun_out/${tag}_rn_step_kernels.txt 2>&1 || true
head -45 gpurun_out/${tag}_rn_step_kernels.txt
GB_VARIANTS=glds128,g128x96,g256x96,p8h2 $S 200 ${tag}_gb.log bin/gemm_bench 20 8192,768,3072,0 8192,768,768,0 8192,2304,768,0 8192,3072,768,0 || exit 1
grep -h '"variant"' gpurun_out/${tag}_gb.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('%-9s %5d %5d %5d L%d %8.1f us %7.1f TF bad=%d rel=%.2e' % (d['variant'],d['M'],d['N'],d['K'],d['layout'],d['us'],d['TF'],d['bad'],d['rel_l2']))"
CLOUD_AMD_CONV_HALO=2 $S 120 ${tag}_cs2.log python bench/conv_shapes.py l1_c2 1024 || exit 1
grep tag gpurun_out/${tag}_cs2.log
echo SESSION_DONE
