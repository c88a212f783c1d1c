#!/usr/bin/env bash
# Round-4 session 39: ResNet-50 knob sweep on the final tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s39}
for r in 1 2; do
$S 240 ${tag}_rn_default_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_XA_WAVES=4 $S 240 ${tag}_rn_xa4_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_GROUPS_MAX=256 $S 240 ${tag}_rn_g256_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_CONV_TALL=0 $S 240 ${tag}_rn_tall0_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_GEMM_PRW=0 $S 240 ${tag}_rn_prw0_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
