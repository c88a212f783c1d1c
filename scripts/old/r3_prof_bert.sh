#!/usr/bin/env bash
# BERT-base b64 kernel trace (serialized weight-gradient stream) + one step's kernel sequence.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s2}
rm -rf gpurun_out/${tag}_prof_bert
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_prof_bert.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_bert -o run --output-format csv -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof_bert adam_kernel > gpurun_out/${tag}_bert_step_kernels.txt
head -60 gpurun_out/${tag}_bert_step_kernels.txt
echo SESSION_DONE
