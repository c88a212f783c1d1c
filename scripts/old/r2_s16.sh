#!/usr/bin/env bash
# Counter pass over a short ResNet-50 run (b256): wait / issue / VALU / MFMA cycles per GEMM shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 60 r2s16_counters.log rocprofv3 -L || exit 1
CLOUD_AMD_WGRAD_STREAM=0 $S 200 r2s16_pmc.log timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv \
  -d gpurun_out/r2s16_pmc -o run --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- python bench.py --via-run 0 --steps 2 --warmup 1 --batch 256 || exit 1
echo SESSION_DONE
