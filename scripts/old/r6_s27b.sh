#!/usr/bin/env bash
# Round-6 session 27b: wide transform-A tiles -- bitwise mode comparison, ResNet fold bitwise
# test under each tile mode.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s27b
$S 300 ${tag}_wide.log python -u -m pytest tests/test_bn_fold_gpu.py -x -q --timeout 200 --timeout-method thread -k "wide_tiles" || exit 1
tail -3 gpurun_out/${tag}_wide.log
for m in 0 1 2; do
CLOUD_AMD_XA_N256=$m $S 300 ${tag}_bitwise_$m.log python -u -m pytest tests/test_bn_fold_gpu.py -x -q --timeout 200 --timeout-method thread -k "resnet_bn_fold_bitwise" || exit 1
tail -1 gpurun_out/${tag}_bitwise_$m.log
done
echo SESSION_DONE
