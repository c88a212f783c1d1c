#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 smallk_bn64.log env CLOUD_AMD_GEMM_TILE_N=64 python bench/smallk_gemm.py || exit 1
$S 300 bench_bn64.log env CLOUD_AMD_GEMM_TILE_N=64 python bench.py --steps 20 --warmup 5 || exit 1
echo SESSION_DONE
