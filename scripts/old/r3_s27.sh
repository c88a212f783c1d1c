#!/usr/bin/env bash
# Round-3 session 27: LayerNorm backward at 8 waves per block (A/B against 4, interleaved; 8 measured
# 6,922-6,934 vs 7,120-7,139 seq/s, ln_bwd 41 us per call, and was removed -- both arms now run the 4-wave kernel),
# BERT kernel breakdown with 8, tuner with the fast worker exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s27}
$S 300 ${tag}_pytest.log python -u -m pytest tests/test_transformer_gpu.py tests/test_bert_hf_parity.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
for i in 1 2 3; do
$S 240 ${tag}_bert_w8_${i}.log python bench/bert_base_synth.py || exit 1
$S 240 ${tag}_bert_w4_${i}.log python bench/bert_base_synth.py || exit 1
done
$S 300 ${tag}_prof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_bert -o run --output-format csv -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof_bert adam_kernel > gpurun_out/${tag}_bert_step_kernels.txt
for i in 1 2; do
$S 300 ${tag}_tuner_${i}.log python bench/tuner_8trials.py || exit 1
done
tail -2 gpurun_out/${tag}_pytest.log
for i in 1 2 3; do echo "bert w8 $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_bert_w8_$i.log) w4 $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_bert_w4_$i.log)"; done
grep -E "ms/step kernel|ln_bwd|ln_fwd|grad_fin" gpurun_out/${tag}_bert_step_kernels.txt | head -6
for i in 1 2; do grep -h '"metric"' gpurun_out/${tag}_tuner_${i}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['wall_s'], max(v['exited'] for v in d['timeline']['workers'].values()))"; done
echo SESSION_DONE
