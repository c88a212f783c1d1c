#!/usr/bin/env bash
# Small-K GEMM occupancy / wait counters (isolated stage-1 1x1-conv GEMMs, bench/smallk_gemm.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 200 smallk.log python bench/smallk_gemm.py || exit 1
$S 120 pmc_occ.log timeout -s KILL 100 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_occ -o run --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -- python bench/smallk_gemm.py || exit 1
echo SESSION_DONE
