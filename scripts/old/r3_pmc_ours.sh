#!/bin/bash
# Counter pass over in-tree GEMM variants only (no torch): usage r3_pmc_ours.sh <tag> <shape> <variants>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
tag=$1; shape=$2; vars=$3
out=gpurun_out/$tag; mkdir -p $out
C="GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
GB_VARIANTS=$vars timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d $out/ours -o ours --output-format csv -- bin/gemm_bench 10 $shape > $out/ours.log 2>&1 || { echo "pmc failed"; tail -20 $out/ours.log; exit 1; }
C2="SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE"
GB_VARIANTS=$vars timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C2 -d $out/ours2 -o ours2 --output-format csv -- bin/gemm_bench 10 $shape > $out/ours2.log 2>&1 || { echo "pmc2 failed"; tail -20 $out/ours2.log; }
python3 scripts/pmc_clock.py $out
python3 scripts/pmc_dump.py $out/ours2
