#!/usr/bin/env bash
# Round-5 session 13: split-K vs 128 x 64 tiles vs hipBLASLt on BERT's N = 768 GEMMs; serialized
# BERT step profile of the current tree; tuner bench (cold value + warm fields).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s13}
$S 200 ${tag}_sk.log python bench/bert_gemm_splitk.py || exit 1
grep '"M"' gpurun_out/${tag}_sk.log
rm -rf gpurun_out/${tag}_bprof
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_bprof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_bprof -o run --output-format csv -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_bprof adam_kernel > gpurun_out/${tag}_bert_step_kernels.txt || true
rm -rf gpurun_out/${tag}_bprof
head -24 gpurun_out/${tag}_bert_step_kernels.txt
$S 400 ${tag}_tuner.log python bench/tuner_8trials.py || exit 1
grep -o '"value": [0-9.]*\|"warm_value": [0-9.]*\|"time_to_best_s": [0-9.]*' gpurun_out/${tag}_tuner.log | tail -3
echo SESSION_DONE
