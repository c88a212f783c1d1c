#!/usr/bin/env bash
# Kernel profile of the b512 ResNet step after the BN-epilogue change.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 400 prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b512 -o run -- python bench.py --steps 6 --warmup 2 || exit 1
echo SESSION_DONE
