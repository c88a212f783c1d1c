#!/usr/bin/env bash
# BERT-base: dense weight-gradient split target sweep + serialized profile with the GEMM shape log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
for i in 1 2; do
  $S 200 r2s22_bert_512_$i.log python bench/bert_base_synth.py --via-run 0 || exit 1
  CLOUD_AMD_DENSE_WGRAD_BLOCKS=256 $S 200 r2s22_bert_256_$i.log python bench/bert_base_synth.py --via-run 0 || exit 1
  CLOUD_AMD_DENSE_WGRAD_BLOCKS=1024 $S 200 r2s22_bert_1024_$i.log python bench/bert_base_synth.py --via-run 0 || exit 1
done
rm -f gpurun_out/r2s22_shapes_bert.jsonl
CLOUD_AMD_WGRAD_STREAM=0 CLOUD_AMD_SHAPE_LOG=gpurun_out/r2s22_shapes_bert.jsonl $S 300 r2s22_prof_bert.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/r2s22_prof_bert -o run -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
echo SESSION_DONE
