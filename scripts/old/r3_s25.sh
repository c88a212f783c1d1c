#!/usr/bin/env bash
# Round-3 session 25: cold-trial attribution for the tuner workers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s25}
$S 200 ${tag}_cold.log python scripts/debug/cold_trial.py || exit 1
CLOUD_AMD_GEMM_LIB=never $S 200 ${tag}_cold_never.log python scripts/debug/cold_trial.py || exit 1
grep -v amdgpu.ids gpurun_out/${tag}_cold_never.log | grep "trial\|import"
echo SESSION_DONE
