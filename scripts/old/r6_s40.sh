#!/usr/bin/env bash
# Round-6 session 40: counters of the stage-3 3x3 implicit-GEMM convolutions (fwd / dgrad / wgrad,
# batch 1024) on the final tree: MFMA busy, wait shares, LDS activity and bank conflicts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s40
$S 120 ${tag}_cs.log python bench/conv_shapes.py l3_c2 1024 || exit 1
cat gpurun_out/${tag}_cs.log | tail -5
out=gpurun_out/${tag}_pmc; mkdir -p $out
C="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
$S 90 ${tag}_pmc1.log timeout -s KILL 80 rocprofv3 --kernel-trace --pmc $C -d $out/p1 -o p1 --output-format csv -- python bench/conv_shapes.py l3_c2 1024 || exit 1
python3 scripts/pmc_clock.py $out > gpurun_out/${tag}_pmc_clock.txt 2>&1 || true
f=$(find $out -name "*counter_collection.csv" | head -1)
python3 scripts/pmc_shapes.py "$f" 20 > gpurun_out/${tag}_pmc_shapes.txt 2>&1 || true
rm -rf $out
head -30 gpurun_out/${tag}_pmc_shapes.txt
echo SESSION_DONE
