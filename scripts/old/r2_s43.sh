#!/usr/bin/env bash
# Counter passes on the final tree (ResNet-50 b256, 2 steps, kernel trace only): wait/issue/MFMA, HBM, LDS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
B="python bench.py --via-run 0 --steps 2 --warmup 1 --batch 256"
CLOUD_AMD_WGRAD_STREAM=0 $S 200 r2s43_pmc1.log timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv \
  -d gpurun_out/r2s43_pmc1 -o run --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- $B || exit 1
CLOUD_AMD_WGRAD_STREAM=0 $S 200 r2s43_pmc2.log timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv \
  -d gpurun_out/r2s43_pmc2 -o run --pmc FETCH_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -- $B || exit 1
CLOUD_AMD_WGRAD_STREAM=0 $S 200 r2s43_pmc3.log timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv \
  -d gpurun_out/r2s43_pmc3 -o run --pmc WRITE_SIZE GRBM_GUI_ACTIVE -- $B || exit 1
echo SESSION_DONE
