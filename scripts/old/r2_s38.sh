#!/usr/bin/env bash
# Re-tune env-level knobs after the split-XCD / batched-epilogue changes (ResNet-50 b1024, BERT b64).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
for i in 1 2; do
  $S 200 r2s38_base_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_BN_APPLY_BLOCKS=2048 $S 200 r2s38_bnab2048_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_WGRAD_BLOCKS=1024 $S 200 r2s38_wb1024_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_WGRAD_BLOCKS=384 $S 200 r2s38_wb384_$i.log python bench.py --via-run 0 || exit 1
done
for i in 1 2; do
  $S 200 r2s38_bert_base_$i.log python bench/bert_base_synth.py --via-run 0 || exit 1
  CLOUD_AMD_DENSE_WGRAD_BLOCKS=1024 $S 200 r2s38_bert_dwb1024_$i.log python bench/bert_base_synth.py --via-run 0 || exit 1
  CLOUD_AMD_DENSE_WGRAD_BLOCKS=256 $S 200 r2s38_bert_dwb256_$i.log python bench/bert_base_synth.py --via-run 0 || exit 1
done
echo SESSION_DONE
