#!/usr/bin/env bash
# Restored tree: full GPU tests, bench, serialized kernel traces of ResNet-50 b1024 and BERT b64
# with the GEMM shape log (scripts/gemm_roofline.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 500 r2s14_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
$S 200 r2s14_bench.log python bench.py || exit 1
rm -f gpurun_out/r2s14_shapes_rn.jsonl gpurun_out/r2s14_shapes_bert.jsonl
CLOUD_AMD_WGRAD_STREAM=0 CLOUD_AMD_SHAPE_LOG=gpurun_out/r2s14_shapes_rn.jsonl $S 300 r2s14_prof_rn.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/r2s14_prof_rn -o run -- python bench.py --via-run 0 --steps 3 --warmup 2 || exit 1
CLOUD_AMD_WGRAD_STREAM=0 CLOUD_AMD_SHAPE_LOG=gpurun_out/r2s14_shapes_bert.jsonl $S 300 r2s14_prof_bert.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/r2s14_prof_bert -o run -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
echo SESSION_DONE
