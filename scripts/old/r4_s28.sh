#!/usr/bin/env bash
# Round-4 session 28: deep fused gradient at depth 2 / 4 with two workgroups per CU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s28}
for d in 1 2 4; do
CLOUD_AMD_XA_DW_DEPTH=$d $S 120 ${tag}_k${d}.log python bench/xa_dw_bench.py || exit 1
done
for d in 1 2 4; do echo "$(grep -o '"depth": "[0-9]"' gpurun_out/${tag}_k$d.log) $(grep -o '"ms": [0-9.]*' gpurun_out/${tag}_k$d.log | tr '\n' ' ') $(grep -o '"dx_repeat_equal": [a-z]*' gpurun_out/${tag}_k$d.log)"; done
echo SESSION_DONE
