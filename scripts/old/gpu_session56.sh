#!/usr/bin/env bash
# End-of-session verification: GPU tests, smoke, headline bench (direct x2 and via run()).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
grep -q "FAILED\|ERROR" gpurun_out/pytest_gpu.log && { echo "gpu tests failed"; exit 1; }
$S 300 smoke.log python __graft_entry__.py smoke || exit 1
for i in 1 2; do $S 300 bench_$i.log python bench.py || exit 1; done
$S 300 bench_via_run.log python bench.py --via-run 1 || exit 1
echo SESSION_DONE
