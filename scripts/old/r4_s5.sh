#!/usr/bin/env bash
# Round-4 session 5: serialized ResNet-50 step profile of the current tree; stock PyTorch-ROCm
# comparators at the headline configs on the same box: HF BERT b64 next to cloud_amd's, then
# ResNet-50 b1024 via run() (channels_last + AMP + MIOpen, torch.optim SGD foreach).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s5}
rm -rf gpurun_out/${tag}_prof_rn
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_prof_rn.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_rn -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof_rn sgd_kernel > gpurun_out/${tag}_rn_step_kernels.txt
rm -rf gpurun_out/${tag}_prof_rn
head -30 gpurun_out/${tag}_rn_step_kernels.txt
$S 240 ${tag}_bert.log python bench/bert_base_synth.py || exit 1
$S 400 ${tag}_stock_bert.log python bench/bert_base_synth.py --stock 1 --steps 20 --warmup 5 || exit 1
$S 240 ${tag}_rn.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 900 ${tag}_stock_rn.log python bench/stock_resnet50.py --gpus 1 --batch 1024 --steps 20 --warmup 5 || exit 1
for f in rn stock_rn bert stock_bert; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log | tail -1)"; done
echo SESSION_DONE
