#!/usr/bin/env bash
# Round-4 session 15: full GPU suite; ResNet-50 with the step pacer (default) vs unbounded
# run-ahead (allocator segments per step in the JSON); BERT dense weight gradients on the
# two-phase 256 core (default) vs the 128 core.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s15}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 600 ${tag}_pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_pytest.log
for i in 1 2; do
$S 240 ${tag}_rn_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_MAX_STEPS_IN_FLIGHT=0 $S 240 ${tag}_rn_nopace_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 240 ${tag}_bert_${i}.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_DENSE_WGRAD_256=0 $S 240 ${tag}_bert_w128_${i}.log python bench/bert_base_synth.py || exit 1
done
tail -1 gpurun_out/${tag}_pytest.log
for f in rn_1 rn_nopace_1 rn_2 rn_nopace_2 bert_1 bert_w128_1 bert_2 bert_w128_2; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log | tail -1)"; done
echo SESSION_DONE
