#!/usr/bin/env bash
# (measured and removed: see docs/performance.md "Round 3"; the switch it A/Bs no longer exists)
# Round-3 session 30: BERT bias gradients from the producing kernels' column sums (the GELU'
# GEMM's statistics epilogue for b1, the fused attention backward for bqkv): numerics tests,
# interleaved A/B against CLOUD_AMD_BERT_BIAS_FROM_EPILOGUE=0, kernel breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s30}
$S 300 ${tag}_pytest.log python -u -m pytest tests/test_transformer_gpu.py tests/test_bert_hf_parity.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
CLOUD_AMD_BERT_BIAS_FROM_EPILOGUE=0 $S 300 ${tag}_pytest_e0.log python -u -m pytest tests/test_bert_hf_parity.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
for i in 1 2 3; do
$S 240 ${tag}_bert_e1_${i}.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_BERT_BIAS_FROM_EPILOGUE=0 $S 240 ${tag}_bert_e0_${i}.log python bench/bert_base_synth.py || exit 1
done
$S 300 ${tag}_prof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_bert -o run --output-format csv -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof_bert adam_kernel > gpurun_out/${tag}_bert_step_kernels.txt
rm -rf gpurun_out/${tag}_prof_bert
tail -1 gpurun_out/${tag}_pytest.log
tail -1 gpurun_out/${tag}_pytest_e0.log
for i in 1 2 3; do echo "bert e1 $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_bert_e1_$i.log) e0 $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_bert_e0_$i.log)"; done
head -24 gpurun_out/${tag}_bert_step_kernels.txt | cut -c1-120
echo SESSION_DONE
