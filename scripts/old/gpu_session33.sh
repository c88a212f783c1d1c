#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 smallk.log python bench/smallk_gemm.py || exit 1
echo SESSION_DONE
