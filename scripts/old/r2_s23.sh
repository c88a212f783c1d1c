#!/usr/bin/env bash
# Re-verify the restored tree: GPU tests, smoke, default bench (via run()), BERT bench,
# and a serialized ResNet-50 b1024 kernel profile with the GEMM shape log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 600 r2s23_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/r2s23_pytest_gpu.log || { echo "GPU tests did not pass"; exit 1; }
$S 200 r2s23_smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S 300 r2s23_bench.log python bench.py || exit 1
$S 200 r2s23_bert.log python bench/bert_base_synth.py --via-run 0 || exit 1
rm -f gpurun_out/r2s23_shapes.jsonl
CLOUD_AMD_WGRAD_STREAM=0 CLOUD_AMD_SHAPE_LOG=gpurun_out/r2s23_shapes.jsonl $S 300 r2s23_prof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/r2s23_prof -o run -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
echo SESSION_DONE
