#!/usr/bin/env bash
# LayerNorm backward row prefetch (reverted LN_BWD_PF switch, BERT) and non-temporal BN backward loads
# (reverted BN_BWD_NT switch, ResNet-50): GPU tests, A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 600 r2s35_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/r2s35_pytest_gpu.log && ! grep -q " failed" gpurun_out/r2s35_pytest_gpu.log || { echo "GPU tests failed"; exit 1; }
LN_BWD_PF=0 $S 600 r2s35_pytest_gpu_pf0.log python -u -m pytest tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
for i in 1 2 3; do
  LN_BWD_PF=0 $S 200 r2s35_bert_pf0_$i.log python bench/bert_base_synth.py --via-run 0 || exit 1
  LN_BWD_PF=1 $S 200 r2s35_bert_pf1_$i.log python bench/bert_base_synth.py --via-run 0 || exit 1
done
for i in 1 2 3; do
  BN_BWD_NT=0 $S 200 r2s35_bench_nt0_$i.log python bench.py --via-run 0 || exit 1
  BN_BWD_NT=1 $S 200 r2s35_bench_nt1_$i.log python bench.py --via-run 0 || exit 1
done
CLOUD_AMD_WGRAD_STREAM=0 $S 300 r2s35_prof_bert.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/r2s35_prof_bert -o run -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
echo SESSION_DONE
