#!/usr/bin/env bash
# Round-3 session 39: the reference workloads on the GPU (single-process and the 2-rank shared-GPU custom loop).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s39}
$S 600 ${tag}_pytest.log python -u -m pytest tests/test_workloads_gpu.py -m gpu -v --timeout 150 --timeout-method thread || exit 1
grep -E "PASSED|FAILED|passed|failed" gpurun_out/${tag}_pytest.log | tail -8
echo SESSION_DONE
