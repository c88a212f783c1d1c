#!/usr/bin/env bash
# Round-5 session 28: one dropout hash per element PAIR (ca_rng.h drop_mul4 in the LayerNorm
# kernels): transformer / attention / BERT GPU tests, BERT x3, serialized BERT step profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s28}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 400 ${tag}_tests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py tests/test_keras_native_gpu.py tests/test_sliced_opt_world1_gpu.py || exit 1
chk ${tag}_tests.log
tail -2 gpurun_out/${tag}_tests.log
for r in 1 2 3; do
$S 200 ${tag}_bert_$r.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
echo "bert_$r $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_bert_$r.log | tail -1)"
done
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_bprof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_bprof -o run --output-format csv -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_bprof adam_kernel > gpurun_out/${tag}_bert_step_kernels.txt || true
rm -rf gpurun_out/${tag}_bprof
head -16 gpurun_out/${tag}_bert_step_kernels.txt
echo SESSION_DONE
