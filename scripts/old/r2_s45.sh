#!/usr/bin/env bash
# GEMM core re-check on the final tree: glds (default) vs glds8 (8 waves, double-buffered) vs pp256.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
for i in 1 2; do
  $S 200 r2s45_glds_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_GEMM_CORE=glds8 $S 200 r2s45_glds8_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_GEMM_CORE=pp256 $S 200 r2s45_pp256_$i.log python bench.py --via-run 0 || exit 1
done
for i in 1 2; do
  $S 200 r2s45_bert_glds_$i.log python bench/bert_base_synth.py --via-run 0 || exit 1
  CLOUD_AMD_GEMM_CORE=glds8 $S 200 r2s45_bert_glds8_$i.log python bench/bert_base_synth.py --via-run 0 || exit 1
done
echo SESSION_DONE
