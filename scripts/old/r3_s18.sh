#!/usr/bin/env bash
# Round-3 session 18: Keras step op attribution on the GPU path, PRW-restricted tree benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s18}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 300 ${tag}_t1.log python -u -m pytest tests/test_gemm_prw_gpu.py tests/test_keras_native_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_t1.log
$S 200 ${tag}_keras_ops.log python scripts/debug/keras_step_ops.py || exit 1
grep -v amdgpu.ids gpurun_out/${tag}_keras_ops.log | head -45
for i in 1 2; do
$S 240 ${tag}_bench_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
done
for f in bench_1 bench_2; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log)"; done
echo SESSION_DONE
