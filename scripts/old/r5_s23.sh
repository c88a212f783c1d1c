#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
scripts/gpu_step.sh 200 r5s23_diag.log python scripts/debug/diag_sliced.py || exit 1
cat gpurun_out/r5s23_diag.log | grep -v amdgpu.ids | head -80
echo SESSION_DONE
