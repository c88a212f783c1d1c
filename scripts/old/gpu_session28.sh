#!/usr/bin/env bash
# Probe: 8-wave double-buffered core (glds8) on the memory-bound small-K ResNet GEMMs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 bench_g8.log env CLOUD_AMD_GEMM_CORE=glds8 python bench.py --steps 20 --warmup 5 || exit 1
$S 400 prof_g8.log env CLOUD_AMD_GEMM_CORE=glds8 CLOUD_AMD_WGRAD_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_g8 -o run -- python bench.py --steps 6 --warmup 2 || exit 1
echo SESSION_DONE
