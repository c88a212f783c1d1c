#!/usr/bin/env bash
# BERT-base: wave-quantisation model of the dense GEMM tile choice (reverted TILE_SLOTS switch) + current kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
for i in 1 2; do
  for t in 1 4 5; do  # TILE_SLOTS: reverted switch (gemm.hip tile_balance slots per CU)
    TILE_SLOTS=$t $S 200 r2s30_bert_slots${t}_$i.log python bench/bert_base_synth.py --via-run 0 || exit 1
  done
done
rm -f gpurun_out/r2s30_shapes_bert.jsonl
CLOUD_AMD_WGRAD_STREAM=0 CLOUD_AMD_SHAPE_LOG=gpurun_out/r2s30_shapes_bert.jsonl $S 300 r2s30_prof_bert.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/r2s30_prof_bert -o run -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
echo SESSION_DONE
