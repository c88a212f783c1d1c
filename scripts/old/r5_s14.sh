#!/usr/bin/env bash
# Round-5 session 14: tile variants on BERT's FFN2 forward (8192 x 768 x 3072 NT).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s14}
GB_VARIANTS=w256x128,glds128,g128x96,p8h2,v256 $S 120 ${tag}_gb.log bin/gemm_bench 30 8192,768,3072,0 8192,768,3072,1 8192,3072,768,0 || exit 1
grep -h '"variant"' gpurun_out/${tag}_gb.log | cut -c1-150
echo SESSION_DONE
