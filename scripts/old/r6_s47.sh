#!/usr/bin/env bash
# Round-6 session 47: GPU idle time per step on the final tree (kernel trace with the weight-gradient
# side stream on; scripts/step_idle.py), ResNet-50 and BERT.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s47
rm -rf gpurun_out/${tag}_r gpurun_out/${tag}_b
$S 300 ${tag}_rprof.log rocprofv3 --kernel-trace -d gpurun_out/${tag}_r -o run --output-format csv -- python bench.py --via-run 0 --steps 6 --warmup 3 || exit 1
python3 scripts/step_idle.py gpurun_out/${tag}_r sgd_kernel > gpurun_out/${tag}_rn_idle.txt || true
rm -rf gpurun_out/${tag}_r
$S 300 ${tag}_bprof.log rocprofv3 --kernel-trace -d gpurun_out/${tag}_b -o run --output-format csv -- python bench/bert_base_synth.py --via-run 0 --steps 8 --warmup 3 || exit 1
python3 scripts/step_idle.py gpurun_out/${tag}_b adam_kernel > gpurun_out/${tag}_bert_idle.txt || true
rm -rf gpurun_out/${tag}_b
head -8 gpurun_out/${tag}_rn_idle.txt gpurun_out/${tag}_bert_idle.txt
echo SESSION_DONE
