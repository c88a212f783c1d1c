#!/usr/bin/env bash
# Round-5 session 20: BERT knob sweep on the current tree (dense weight-gradient split target,
# prefetching dense epilogue), interleaved, two runs each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s20}
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
$S 400 ${tag}_t.log $PT tests/test_transformer_gpu.py tests/test_kernels_gpu.py tests/test_bert_hf_parity.py tests/test_keras_native_gpu.py || exit 1
grep -q "FAILED\|Error" gpurun_out/${tag}_t.log && { echo T_FAILED; tail -40 gpurun_out/${tag}_t.log; exit 1; }
tail -2 gpurun_out/${tag}_t.log
for r in 1 2; do
for b in 640 256 384 1024; do
CLOUD_AMD_DENSE_WGRAD_BLOCKS=$b $S 200 ${tag}_b${b}_$r.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
done
CLOUD_AMD_EPI_PF=0 $S 200 ${tag}_pf0_$r.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_LN_BWD16=0 $S 200 ${tag}_ln4_$r.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
rm -rf gpurun_out/${tag}_bprof
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_bprof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_bprof -o run --output-format csv -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_bprof adam_kernel > gpurun_out/${tag}_bert_step_kernels.txt || true
rm -rf gpurun_out/${tag}_bprof
head -20 gpurun_out/${tag}_bert_step_kernels.txt
echo SESSION_DONE
