#!/usr/bin/env bash
# Round-3 session 1: GPU tests + smoke on the tree with the 256 GEMM core, then the GEMM
# core A/B (auto vs 128-only) and the two headline benches with each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
mode=${1:-all}
if [ "$mode" = all ] || [ "$mode" = tests ]; then
  $S 700 r3s1_pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
  grep -q " passed" gpurun_out/r3s1_pytest_gpu.log && ! grep -qE " failed| error" gpurun_out/r3s1_pytest_gpu.log || { echo "GPU tests failed"; tail -40 gpurun_out/r3s1_pytest_gpu.log; exit 1; }
  $S 200 r3s1_smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
if [ "$mode" = all ] || [ "$mode" = bench ]; then
  $S 240 r3s1_gemm_ab_auto.log python bench/gemm_core_ab.py || exit 1
  CLOUD_AMD_GEMM_CORE=glds $S 240 r3s1_gemm_ab_glds.log python bench/gemm_core_ab.py || exit 1
  $S 240 r3s1_bench.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
  CLOUD_AMD_GEMM_CORE=glds $S 240 r3s1_bench_glds.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
  $S 240 r3s1_bert.log python bench/bert_base_synth.py || exit 1
fi
echo SESSION_DONE
