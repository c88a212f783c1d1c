#!/usr/bin/env bash
# (measured and removed: the CLOUD_AMD_BN_NT switch no longer exists; see docs/performance.md "Round 3")
# Round-3 session 34: non-temporal loads / stores in the BatchNorm apply passes
# (CLOUD_AMD_BN_NT 0 / 1 / 3): per-shape bandwidth, then ResNet-50 end to end, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s34}
$S 300 ${tag}_pytest.log python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "bn or batchnorm" || exit 1
for nt in 0 1 3; do
CLOUD_AMD_BN_NT=$nt $S 300 ${tag}_bnbw_nt${nt}.log python bench/bn_apply_bw.py || exit 1
done
for i in 1 2 3; do
for nt in 0 1 3; do
CLOUD_AMD_BN_NT=$nt $S 240 ${tag}_bench_nt${nt}_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
done
done
tail -1 gpurun_out/${tag}_pytest.log
for nt in 0 1 3; do echo "== nt$nt"; grep -v amdgpu.ids gpurun_out/${tag}_bnbw_nt${nt}.log | tail -20 | cut -c1-160; done
for i in 1 2 3; do echo "rn $(for nt in 0 1 3; do echo -n "nt$nt $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_bench_nt${nt}_$i.log | tail -1)  "; done)"; done
echo SESSION_DONE
