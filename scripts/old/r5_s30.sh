#!/usr/bin/env bash
# Round-5 session 30: BatchNorm statistics finalize group size (CLOUD_AMD_BN_FIN_RPG 512 default /
# 256 / 128), BN finalize tests, ResNet-50 interleaved, three runs each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s30}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
for r in 512 128; do
CLOUD_AMD_BN_FIN_RPG=$r $S 300 ${tag}_t$r.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_finalize_gpu.py tests/test_kernels_gpu.py || exit 1
chk ${tag}_t$r.log
done
run() { local name=$1; shift; env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_${name}.log 2>&1 || { echo "fail $name"; exit 1; }; echo "$name $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_${name}.log | tail -1)"; }
for i in 1 2 3; do
run r512_$i CLOUD_AMD_BN_FIN_RPG=512
run r256_$i CLOUD_AMD_BN_FIN_RPG=256
run r128_$i CLOUD_AMD_BN_FIN_RPG=128
done
echo SESSION_DONE
