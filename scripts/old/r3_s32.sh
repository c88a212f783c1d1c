#!/usr/bin/env bash
# (measured and removed: see docs/performance.md "Round 3"; the switch it A/Bs no longer exists)
# Round-3 session 32 (NN statistics epilogue accumulated in registers): same-box kernel breakdowns with / without the BERT bias gradients from
# the producing kernels' column sums (side stream off: serialized kernel times), plus interleaved pairs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s32}
$S 300 ${tag}_pytest.log python -u -m pytest tests/test_transformer_gpu.py tests/test_bert_hf_parity.py tests/test_keras_native_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
tail -1 gpurun_out/${tag}_pytest.log
for e in 1 0; do
CLOUD_AMD_WGRAD_STREAM=0 CLOUD_AMD_BERT_BIAS_FROM_EPILOGUE=$e $S 300 ${tag}_prof_e$e.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_bert_e$e -o run --output-format csv -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof_bert_e$e adam_kernel > gpurun_out/${tag}_bert_step_kernels_e$e.txt
rm -rf gpurun_out/${tag}_prof_bert_e$e
done
for i in 1 2 3 4; do
$S 240 ${tag}_bert_e1_${i}.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_BERT_BIAS_FROM_EPILOGUE=0 $S 240 ${tag}_bert_e0_${i}.log python bench/bert_base_synth.py || exit 1
done
for i in 1 2 3 4; do echo "bert e1 $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_bert_e1_$i.log) e0 $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_bert_e0_$i.log)"; done
for e in 1 0; do echo "== e$e"; head -14 gpurun_out/${tag}_bert_step_kernels_e$e.txt | cut -c1-110; done
echo SESSION_DONE
