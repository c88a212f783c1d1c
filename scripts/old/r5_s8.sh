#!/usr/bin/env bash
# Round-5 session 8: counters of the LDS-resident 3x3 convolution (stage-1 shape, batch 1024),
# halo on / off timing, the one-launch BatchNorm finalize test and a ResNet-50 A/B of it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s8}
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$S 200 ${tag}_fin.log $PT tests/test_bn_finalize_gpu.py tests/test_conv_halo_gpu.py || exit 1
grep -q "FAILED\|Error" gpurun_out/${tag}_fin.log && { echo FIN_FAILED; tail -30 gpurun_out/${tag}_fin.log; exit 1; }
$S 120 ${tag}_cs_h1.log python bench/conv_shapes.py l1_c2 1024 || exit 1
CLOUD_AMD_CONV_HALO=0 $S 120 ${tag}_cs_h0.log python bench/conv_shapes.py l1_c2 1024 || exit 1
cat gpurun_out/${tag}_cs_h1.log gpurun_out/${tag}_cs_h0.log
out=gpurun_out/${tag}_pmc; mkdir -p $out
C="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
$S 90 ${tag}_pmc1.log timeout -s KILL 80 rocprofv3 --kernel-trace --pmc $C -d $out/p1 -o p1 --output-format csv -- python bench/conv_shapes.py l1_c2 1024 || exit 1
C2="GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVES"
$S 90 ${tag}_pmc2.log timeout -s KILL 80 rocprofv3 --kernel-trace --pmc $C2 -d $out/p2 -o p2 --output-format csv -- python bench/conv_shapes.py l1_c2 1024 || exit 1
python3 scripts/pmc_clock.py $out > gpurun_out/${tag}_pmc_clock.txt 2>&1 || true
python3 scripts/pmc_dump.py $out/p2 > gpurun_out/${tag}_pmc_dump.txt 2>&1 || true
grep -i "halo\|conv_glds" gpurun_out/${tag}_pmc_clock.txt | head -20
grep -i "halo\|conv_glds" gpurun_out/${tag}_pmc_dump.txt | head -20
CLOUD_AMD_BN_FIN_MERGED=0 $S 200 ${tag}_rn_f0.log python bench.py --steps 20 --warmup 5 || exit 1
$S 200 ${tag}_rn_f1.log python bench.py --steps 20 --warmup 5 || exit 1
for f in gpurun_out/${tag}_rn_f*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
