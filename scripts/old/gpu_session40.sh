#!/usr/bin/env bash
# PMC counter passes (one block set per pass, kernel trace only) on a short ResNet-50 run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
ARGS="python bench.py --steps 2 --warmup 1 --batch 256"
$S 120 pmc_sq.log timeout -s KILL 100 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_sq -o run --pmc SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -- $ARGS || exit 1
$S 120 pmc_fetch.log timeout -s KILL 100 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run --pmc FETCH_SIZE -- $ARGS || exit 1
$S 120 pmc_write.log timeout -s KILL 100 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run --pmc WRITE_SIZE -- $ARGS || exit 1
echo SESSION_DONE
