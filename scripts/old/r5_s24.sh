#!/usr/bin/env bash
# Round-5 session 24: ResNet-50 knob sweep on the current tree (weight-gradient split targets,
# BN apply grid, fold sites), interleaved, two runs each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s24}
run() { local name=$1; shift; env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_${name}.log 2>&1 || { echo "fail $name"; exit 1; }; echo "$name $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_${name}.log | tail -1)"; }
for r in 1 2; do
run base_$r CLOUD_AMD_WGRAD_BLOCKS=512
run wg256_$r CLOUD_AMD_WGRAD_BLOCKS=256
run wg1024_$r CLOUD_AMD_WGRAD_BLOCKS=1024
run wgs256_$r CLOUD_AMD_WGRAD_BLOCKS_SMALLM=256
run wgs1024_$r CLOUD_AMD_WGRAD_BLOCKS_SMALLM=1024
run ab1024_$r CLOUD_AMD_BN_APPLY_BLOCKS=1024
run ab4096_$r CLOUD_AMD_BN_APPLY_BLOCKS=4096
run fold256_$r CLOUD_AMD_BN_FOLD_MAX_N=256
done
echo SESSION_DONE
