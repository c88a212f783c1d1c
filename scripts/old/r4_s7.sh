#!/usr/bin/env bash
# Round-4 session 7: 8-phase 256 core with three half tiles in flight (vmcnt(6)): numerics,
# then GEMM core A/B (ring vs p8) interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s7}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 300 ${tag}_g256_tests.log python -u -m pytest tests/test_gemm256_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_g256_tests.log
for i in 1 2; do
$S 300 ${tag}_gemm_ring_${i}.log python bench/gemm_core_ab.py || exit 1
CLOUD_AMD_GEMM_CORE=p8 $S 300 ${tag}_gemm_p8_${i}.log python bench/gemm_core_ab.py || exit 1
done
grep -h summary gpurun_out/${tag}_gemm_*.log
echo SESSION_DONE
