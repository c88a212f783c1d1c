#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 pytest_ddp_gpu.log python -m pytest tests/test_ddp_gpu.py -q || exit 1
$S 300 graph_probe.log python scripts/graph_probe.py || exit 1
echo SESSION_DONE
