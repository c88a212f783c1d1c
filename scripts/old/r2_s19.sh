#!/usr/bin/env bash
# Core A/B after the loader rewrite: 4-wave single-stage (default) vs 8-wave double-buffered (glds8).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
for i in 1 2; do
  $S 200 r2s19_glds_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_GEMM_CORE=glds8 $S 200 r2s19_glds8_$i.log python bench.py --via-run 0 || exit 1
done
CLOUD_AMD_GEMM_CORE=glds8 $S 200 r2s19_bert_glds8.log python bench/bert_base_synth.py --via-run 0 || exit 1
$S 200 r2s19_bert_glds.log python bench/bert_base_synth.py --via-run 0 || exit 1
echo SESSION_DONE
