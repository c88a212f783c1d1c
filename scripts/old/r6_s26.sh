#!/usr/bin/env bash
# Round-6 session 26: sparse projection-shortcut input gradient (no zero-fill) -- kernel tests,
# ResNet-50 A/B (CLOUD_AMD_DS_SPARSE_DGRAD on/off, interleaved).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s26
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 400 ${tag}_kt.log python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "sparse or fused_bottleneck or dgrad" || exit 1
chk ${tag}_kt.log
tail -2 gpurun_out/${tag}_kt.log
for r in 1 2; do
CLOUD_AMD_DS_SPARSE_DGRAD=1 $S 200 ${tag}_rn_on_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_DS_SPARSE_DGRAD=0 $S 200 ${tag}_rn_off_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
