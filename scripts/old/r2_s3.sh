#!/usr/bin/env bash
# Serialized ResNet-50 b512 kernel profile (weight-gradient stream off) for per-shape attribution.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
CLOUD_AMD_WGRAD_STREAM=0 $S 300 r2s3_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/r2s3_prof -o run -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
echo SESSION_DONE
