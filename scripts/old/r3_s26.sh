#!/usr/bin/env bash
# Round-3 session 26: cold trial after the engine-direct seeded backward (no sympy import)
# and the fused evaluate; tuner with the timeline; Keras GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s26}
$S 200 ${tag}_cold.log python scripts/debug/cold_trial.py || exit 1
$S 300 ${tag}_pytest.log python -u -m pytest tests/test_keras_native_gpu.py tests/test_transformer_gpu.py tests/test_bert_hf_parity.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
for i in 1 2 3; do
$S 300 ${tag}_tuner_${i}.log python bench/tuner_8trials.py || exit 1
$S 240 ${tag}_bert_lnb1_${i}.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_LN_BIAS_FWD=0 $S 240 ${tag}_bert_lnb0_${i}.log python bench/bert_base_synth.py || exit 1
done
for i in 1 2 3; do echo "bert lnb1 $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_bert_lnb1_$i.log) lnb0 $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_bert_lnb0_$i.log)"; done
tail -2 gpurun_out/${tag}_pytest.log
grep -v amdgpu.ids gpurun_out/${tag}_cold.log | grep "trial\|import"
for i in 1 2 3; do grep -h '"metric"' gpurun_out/${tag}_tuner_${i}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['wall_s']); [print(k, v) for k, v in d['timeline']['workers'].items()]; [print(t) for t in d['timeline']['trials']]"; done
echo SESSION_DONE
