#!/usr/bin/env bash
# Round-3 session 29: startup phases of run()->first step on the driver's command; the new
# Keras evaluate GPU test; BERT.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s29}
$S 300 ${tag}_pytest.log python -u -m pytest tests/test_keras_native_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
for i in 1 2; do
$S 240 ${tag}_bench_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 240 ${tag}_bert_${i}.log python bench/bert_base_synth.py || exit 1
done
tail -1 gpurun_out/${tag}_pytest.log
for f in bench_1 bert_1 bench_2 bert_2; do grep -h '"metric"' gpurun_out/${tag}_$f.log | grep -v "^\[chief" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['run_to_first_step_s'], d['startup_phases_rank0'])"; done
echo SESSION_DONE
