#!/usr/bin/env bash
# 256x256 ping-pong GEMM variants: TFLOP/s at 4096^3 and BERT FFN shapes, plus one counter
# pass per core on the 4096^3 forward GEMM (kernel trace only; no trace domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
for c in glds pp256; do
  CLOUD_AMD_GEMM_CORE=$c $S 60 r2s12_one_$c.log python bench/gemm_one.py 4096 4096 4096 --iters 50 || exit 1
  CLOUD_AMD_GEMM_CORE=$c $S 60 r2s12_one8k_$c.log python bench/gemm_one.py 8192 8192 8192 --iters 10 || exit 1
  CLOUD_AMD_GEMM_CORE=$c $S 60 r2s12_ffn1_$c.log python bench/gemm_one.py 32768 3072 768 --iters 50 || exit 1
done
for c in pp256; do
  CLOUD_AMD_GEMM_CORE=$c $S 120 r2s12_pmc_$c.log timeout -s KILL 100 rocprofv3 --kernel-trace --output-format csv \
    -d gpurun_out/r2s12_pmc_$c -o run --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS \
    SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE -- python bench/gemm_one.py 4096 4096 4096 --iters 10 || exit 1
done
CLOUD_AMD_GEMM_CORE=pp256 $S 200 r2s12_ab_pp256.log python bench/gemm_core_ab.py || exit 1
echo SESSION_DONE
