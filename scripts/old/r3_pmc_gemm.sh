#!/bin/bash
# Counter pass (kernel trace + PMC, no sys/runtime trace): clock (GRBM_GUI_ACTIVE / 8 / wall),
# MFMA busy and wave-state split of the in-tree GEMM cores vs hipBLASLt on one shape.
# usage: scripts/r3_pmc_gemm.sh <tag> <M,N,K,layout> [variants]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
tag=$1; shape=$2; vars=${3:-v4r_256,v3_256,glds128}
out=gpurun_out/$tag; mkdir -p $out
C="GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
GB_VARIANTS=$vars timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d $out/ours -o ours --output-format csv -- bin/gemm_bench 10 $shape > $out/ours.log 2>&1 || { echo "ours pmc failed"; tail -20 $out/ours.log; exit 1; }
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C -d $out/blas -o blas --output-format csv -- python3 bench/blas_ref.py $shape > $out/blas.log 2>&1 || { echo "blas pmc failed"; tail -20 $out/blas.log; exit 1; }
python3 scripts/pmc_clock.py $out
