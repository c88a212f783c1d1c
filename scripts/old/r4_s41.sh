#!/usr/bin/env bash
# Round-4 session 41: layer-1 3x3 / stem weight gradients on 64 x 64 tiles (CLOUD_AMD_WGRAD_N64).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s41}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
CLOUD_AMD_WGRAD_N64=1 $S 300 ${tag}_conv.log python -u -m pytest tests/test_kernels_gpu.py tests/test_stem_tail_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_conv.log
for r in 1 2; do
$S 240 ${tag}_rn_default_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_WGRAD_N64=1 $S 240 ${tag}_rn_n64_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
done
tail -1 gpurun_out/${tag}_conv.log
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
