#!/usr/bin/env bash
# Round-2 GPU session: GPU tests, smoke, headline bench, kernel profile.
# usage: scripts/r2_session.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-s1}
S=scripts/gpu_step.sh
$S 300 ${tag}_pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
$S 200 ${tag}_smoke.log python __graft_entry__.py smoke || exit 1
$S 200 ${tag}_bench.log python bench.py || exit 1
$S 300 ${tag}_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run -- python bench.py --steps 5 --warmup 3 || exit 1
echo SESSION_DONE
