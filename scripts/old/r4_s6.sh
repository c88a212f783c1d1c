#!/usr/bin/env bash
# Round-4 session 6: BN-fold site policy A/B on ResNet-50 (off / N<=64 / N<=512 / every site),
# interleaved, plus the fold tests under the policy knobs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s6}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 300 ${tag}_fold_tests.log python -u -m pytest tests/test_bn_fold_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_fold_tests.log
for i in 1 2; do
CLOUD_AMD_BN_FOLD=0 CLOUD_AMD_BN_FOLD_FWD=0 $S 240 ${tag}_off_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 240 ${tag}_n64_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD_MAX_N=512 $S 240 ${tag}_n512_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD_ALL=1 $S 240 ${tag}_all_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
done
for f in off_1 n64_1 n512_1 all_1 off_2 n64_2 n512_2 all_2; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log | tail -1)"; done
echo SESSION_DONE
