#!/usr/bin/env bash
# Native input pipeline: GPU tests + throughput (host loader, device loader, loader-fed ResNet-50).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "FAILED\|ERROR" gpurun_out/pytest_gpu.log && { echo "gpu tests failed"; exit 1; }
$S 400 input_pipeline.log python bench/input_pipeline.py --images 6144 || exit 1
rm -rf /tmp/cloud_amd_synth_imagenet
echo SESSION_DONE
