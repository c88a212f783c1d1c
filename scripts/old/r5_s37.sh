#!/usr/bin/env bash
# Round-5 session 37: deterministic token-type embedding gradient (block-ordered reduction):
# transformer / sliced-optimizer (now bitwise over 3 BERT steps) / Keras GPU tests, BERT x2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s37}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 400 ${tag}_t.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py tests/test_sliced_opt_world1_gpu.py tests/test_keras_native_gpu.py tests/test_ctl_gpu.py || exit 1
chk ${tag}_t.log
tail -1 gpurun_out/${tag}_t.log
for r in 1 2; do
$S 200 ${tag}_bert_$r.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
echo "bert_$r $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_bert_$r.log | tail -1)"
done
rm -rf gpurun_out/${tag}_bprof
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_bprof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_bprof -o run --output-format csv -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_bprof adam_kernel > gpurun_out/${tag}_bert_step_kernels.txt || true
rm -rf gpurun_out/${tag}_bprof
grep -E "embed|kernel time" gpurun_out/${tag}_bert_step_kernels.txt | head -6
echo SESSION_DONE
