#!/usr/bin/env bash
# A/B on one box: BERT with / without the LN-fused bias sums, alternating, 3 runs each; ResNet x2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
for i in 1 2 3; do
  CLOUD_AMD_LN_BIAS_SUM=1 $S 200 ab_bert_on_$i.log python bench/bert_base_synth.py --via-run 0 || exit 1
  CLOUD_AMD_LN_BIAS_SUM=0 $S 200 ab_bert_off_$i.log python bench/bert_base_synth.py --via-run 0 || exit 1
done
$S 200 ab_resnet_1.log python bench.py --via-run 0 || exit 1
$S 200 ab_resnet_2.log python bench.py --via-run 0 || exit 1
echo SESSION_DONE
