#!/usr/bin/env bash
# Round-4 session 26: deep-stream fused input+weight gradient (CLOUD_AMD_XA_DW_DEPTH):
# numerics, kernel A/B at the stage-1 shape, ResNet-50 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s26}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 300 ${tag}_fold.log python -u -m pytest tests/test_bn_fold_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_fold.log
for d in 0 1 2 4; do
CLOUD_AMD_XA_DW_DEPTH=$d $S 120 ${tag}_k${d}.log python bench/xa_dw_bench.py || exit 1
done
for r in 1 2; do
for d in 2 0; do
CLOUD_AMD_XA_DW_DEPTH=$d $S 240 ${tag}_rn_d${d}_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
done
done
tail -1 gpurun_out/${tag}_fold.log
for d in 0 1 2 4; do tail -1 gpurun_out/${tag}_k${d}.log; done
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
