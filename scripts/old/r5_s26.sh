#!/usr/bin/env bash
# Round-5 session 26: the 4-wave, one-barrier-per-K-tile 256 x 128 GEMM core (ca_gemm256w4.h)
# against the two-phase 256 core and the 128 core, square and BERT shapes, all layouts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s26}
GB_VARIANTS=w4x128,p8h2,glds128 $S 300 ${tag}_gb.log bin/gemm_bench 20 4096,4096,4096,0 8192,8192,8192,0 4096,4096,4096,1 4096,4096,4096,2 8192,2304,768,0 8192,3072,768,0 8192,768,3072,0 8192,768,3072,1 8192,3072,768,1 768,3072,8192,2 || exit 1
cat gpurun_out/${tag}_gb.log
echo SESSION_DONE
