#!/usr/bin/env bash
# Round-5 session 15: 256 x 256 two-phase core vs the 128 core on ResNet-50's 1x1 input-gradient
# shapes (NN) at batch 1024, and their forward (NT) shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s15}
GB_VARIANTS=p8h2,glds128,w256x128 $S 200 ${tag}_gb.log bin/gemm_bench 10 200704,256,1024,1 50176,512,2048,1 802816,128,512,1 200704,1024,256,1 50176,2048,512,1 802816,512,128,1 200704,1024,256,0 50176,2048,512,0 || exit 1
grep -h '"variant"' gpurun_out/${tag}_gb.log | cut -c1-150
echo SESSION_DONE
