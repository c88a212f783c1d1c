#!/usr/bin/env bash
# Round-5 session 19: current tree -- BERT and ResNet-50 benches (3 runs each, interleaved),
# serialized BERT and ResNet step profiles, epilogue costs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s19}
for r in 1 2 3; do
$S 200 ${tag}_bert_$r.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
$S 200 ${tag}_rn_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_bert_*.log gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
$S 200 ${tag}_epi.log python bench/dense_epilogue_cost.py || exit 1
grep case gpurun_out/${tag}_epi.log
rm -rf gpurun_out/${tag}_bprof gpurun_out/${tag}_rprof
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_bprof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_bprof -o run --output-format csv -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_bprof adam_kernel > gpurun_out/${tag}_bert_step_kernels.txt || true
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_rprof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_rprof -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_rprof sgd_kernel > gpurun_out/${tag}_rn_step_kernels.txt || true
rm -rf gpurun_out/${tag}_bprof gpurun_out/${tag}_rprof
head -14 gpurun_out/${tag}_bert_step_kernels.txt
head -3 gpurun_out/${tag}_rn_step_kernels.txt
echo SESSION_DONE
