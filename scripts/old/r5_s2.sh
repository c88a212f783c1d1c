#!/usr/bin/env bash
# Round-5 session 2: serialized (weight-gradient stream off) step profiles of BERT and ResNet-50
# on the current tree; BERT bench with the ready-ordered buckets (overlap budget).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s2}
rm -rf gpurun_out/${tag}_bprof gpurun_out/${tag}_rprof
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_bprof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_bprof -o run --output-format csv -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_bprof adam_kernel > gpurun_out/${tag}_bert_step_kernels.txt || true
rm -rf gpurun_out/${tag}_bprof
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_rprof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_rprof -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_rprof sgd_kernel > gpurun_out/${tag}_rn_step_kernels.txt || true
rm -rf gpurun_out/${tag}_rprof
$S 300 ${tag}_bert.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
head -40 gpurun_out/${tag}_bert_step_kernels.txt
head -30 gpurun_out/${tag}_rn_step_kernels.txt
grep -o '"overlap_budget".*' gpurun_out/${tag}_bert.log | head -c 1500; echo
echo SESSION_DONE
