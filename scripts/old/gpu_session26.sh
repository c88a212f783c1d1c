#!/usr/bin/env bash
# Serialized (no wgrad side stream) kernel profiles, BN epilogue on / off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export CLOUD_AMD_WGRAD_STREAM=0
S=scripts/gpu_step.sh
$S 400 prof_e1.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ser_e1 -o run -- python bench.py --steps 6 --warmup 2 || exit 1
export CLOUD_AMD_BN_BWD_EPILOGUE=0
$S 400 prof_e0.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ser_e0 -o run -- python bench.py --steps 6 --warmup 2 || exit 1
echo SESSION_DONE
