#!/usr/bin/env bash
# Round-6 session 23: ResNet fused block with the side-stream join deferred one block -- block
# tests, ResNet A/B x3 interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s23
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
CLOUD_AMD_RN_DEFER_JOIN=1 $S 600 ${tag}_t.log python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bn_fold_gpu.py tests/test_kernels_gpu.py tests/test_ddp_gpu.py tests/test_sliced_opt_world1_gpu.py tests/test_rccl_dataplane_gpu.py || exit 1
chk ${tag}_t.log
tail -1 gpurun_out/${tag}_t.log
for r in 1 2 3; do
$S 200 ${tag}_rn_base_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_RN_DEFER_JOIN=1 $S 200 ${tag}_rn_defer_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
