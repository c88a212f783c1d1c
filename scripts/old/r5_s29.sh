#!/usr/bin/env bash
# Round-5 session 29: tile shapes for BERT's N = 768 forwards (FFN2 8192x768x3072, attention
# output 8192x768x768) in one process: 128x64 (dispatched), 128x96, 128x128, 256x96.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s29}
GB_VARIANTS=g128x64,g128x96,glds128,g256x96 $S 200 ${tag}_gb.log bin/gemm_bench 30 8192,768,3072,0 8192,768,768,0 8192,768,3072,1 8192,768,768,1 8192,768,2304,1 || exit 1
cat gpurun_out/${tag}_gb.log
echo SESSION_DONE
