#!/usr/bin/env bash
# 256x256 GEMM core (CLOUD_AMD_GEMM_CORE=g256) vs the 128x128 glds core: correctness and
# TFLOP/s on the BERT / ResNet / 4096^3 shapes, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
CLOUD_AMD_GEMM_CORE=pp256 $S 200 r2s11_gemm_pp256.log python bench/gemm_core_ab.py || exit 1
CLOUD_AMD_GEMM_CORE=glds $S 200 r2s11_gemm_glds.log python bench/gemm_core_ab.py || exit 1
echo SESSION_DONE
