#!/usr/bin/env bash
# GEMM cores vs hipBLASLt on BERT / ResNet shapes; BERT serialized profile; HF parity GPU test; tuner bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 200 r2s6_hf_parity.log python -u -m pytest tests/test_bert_hf_parity.py tests/test_keras_native_gpu.py -m gpu -v --timeout 120 --timeout-method thread || exit 1
$S 200 r2s6_gemm_ab.log python bench/gemm_core_ab.py || exit 1
CLOUD_AMD_WGRAD_STREAM=0 $S 300 r2s6_bert_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/r2s6_bert -o run -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
$S 400 r2s6_tuner.log python bench/tuner_8trials.py || exit 1
echo SESSION_DONE
