#!/usr/bin/env bash
# Round-6 session 42: CLOUD_AMD_CONV_RP on the 3x3 weight gradients only -- ResNet-50 A/B interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s42
CLOUD_AMD_CONV_RP=1 $S 300 ${tag}_kt.log python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv or fused_bottleneck" || exit 1
tail -1 gpurun_out/${tag}_kt.log
for r in 1 2 3; do
$S 200 ${tag}_rn_off_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_CONV_RP=1 $S 200 ${tag}_rn_on_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
