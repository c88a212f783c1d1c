#!/usr/bin/env bash
# Batched-LDS-read epilogue for forward dense GEMMs (CLOUD_AMD_EPI_PF): GPU tests, ResNet/BERT A/B, profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
CLOUD_AMD_EPI_PF=1 $S 600 r2s36_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/r2s36_pytest_gpu.log && ! grep -q " failed" gpurun_out/r2s36_pytest_gpu.log || { echo "GPU tests failed"; exit 1; }
for i in 1 2 3; do
  CLOUD_AMD_EPI_PF=0 $S 200 r2s36_bench_pf0_$i.log python bench.py --via-run 0 || exit 1
  CLOUD_AMD_EPI_PF=1 $S 200 r2s36_bench_pf1_$i.log python bench.py --via-run 0 || exit 1
done
for i in 1 2; do
  CLOUD_AMD_EPI_PF=0 $S 200 r2s36_bert_pf0_$i.log python bench/bert_base_synth.py --via-run 0 || exit 1
  CLOUD_AMD_EPI_PF=1 $S 200 r2s36_bert_pf1_$i.log python bench/bert_base_synth.py --via-run 0 || exit 1
done
rm -f gpurun_out/r2s36_shapes.jsonl
CLOUD_AMD_EPI_PF=1 CLOUD_AMD_WGRAD_STREAM=0 CLOUD_AMD_SHAPE_LOG=gpurun_out/r2s36_shapes.jsonl $S 300 r2s36_prof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/r2s36_prof -o run -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
echo SESSION_DONE
