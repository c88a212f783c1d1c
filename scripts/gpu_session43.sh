#!/usr/bin/env bash
# BN group-reduce + finalize merged via last-block tickets: tests, A/B x2, serialized profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "FAILED\|ERROR" gpurun_out/pytest_gpu.log && { echo "gpu tests failed"; exit 1; }
for i in 1 2; do
  $S 300 bench_t1_$i.log python bench.py --steps 20 --warmup 5 || exit 1
  $S 300 bench_t0_$i.log env CLOUD_AMD_BN_TICKETS=0 python bench.py --steps 20 --warmup 5 || exit 1
done
$S 400 prof.log env CLOUD_AMD_WGRAD_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ser6 -o run -- python bench.py --steps 6 --warmup 2 || exit 1
echo SESSION_DONE
