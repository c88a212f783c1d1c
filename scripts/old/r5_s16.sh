#!/usr/bin/env bash
# Round-5 session 16: dense-layer epilogue costs on BERT's FFN shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s16}
$S 200 ${tag}_epi.log python bench/dense_epilogue_cost.py || exit 1
grep case gpurun_out/${tag}_epi.log
echo SESSION_DONE
