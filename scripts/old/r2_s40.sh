#!/usr/bin/env bash
# Attention backward: dK/dV and dQ in one launch (reverted ATTN_BWD_FUSED switch, attn.hip): GPU tests, BERT A/B, profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 600 r2s40_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/r2s40_pytest_gpu.log && ! grep -q " failed" gpurun_out/r2s40_pytest_gpu.log || { echo "GPU tests failed"; exit 1; }
ATTN_BWD_FUSED=0 $S 300 r2s40_pytest_transformer_unfused.log python -u -m pytest tests/test_transformer_gpu.py tests/test_bert_hf_parity.py -x -q --timeout 120 --timeout-method thread || exit 1
for i in 1 2 3; do
  ATTN_BWD_FUSED=0 $S 200 r2s40_bert_f0_$i.log python bench/bert_base_synth.py --via-run 0 || exit 1
  ATTN_BWD_FUSED=1 $S 200 r2s40_bert_f1_$i.log python bench/bert_base_synth.py --via-run 0 || exit 1
done
CLOUD_AMD_WGRAD_STREAM=0 $S 300 r2s40_prof_bert.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/r2s40_prof_bert -o run -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
echo SESSION_DONE
