#!/usr/bin/env bash
# Transposed-accumulator epilogue: GPU tests, bench x2, serialized profile, GEMM A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r2s8}
$S 400 ${tag}_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/${tag}_pytest_gpu.log && ! grep -q "FAILED\|ERROR" gpurun_out/${tag}_pytest_gpu.log || { echo "gpu tests failed"; exit 1; }
$S 200 ${tag}_bench_1.log python bench.py || exit 1
$S 200 ${tag}_bench_2.log python bench.py || exit 1
$S 200 ${tag}_bert.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
$S 200 ${tag}_gemm_ab.log python bench/gemm_core_ab.py || exit 1
echo SESSION_DONE
