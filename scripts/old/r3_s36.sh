#!/usr/bin/env bash
# Round-3 session 36: the final tree (re-check after the last changes) -- the driver's round-end checks (smoke, full GPU suite,
# bench command), the ResNet-50 batch sweep (b256 / b512 / b1024) of the same tree, BERT, tuner.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s36}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 300 ${tag}_smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S 900 ${tag}_pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_pytest.log
for i in 1; do
$S 240 ${tag}_bench_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 240 ${tag}_rn_b512_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 --batch 512 || exit 1
$S 240 ${tag}_rn_b256_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 --batch 256 || exit 1
$S 240 ${tag}_bert_${i}.log python bench/bert_base_synth.py || exit 1
$S 300 ${tag}_tuner_${i}.log python bench/tuner_8trials.py || exit 1
done
tail -1 gpurun_out/${tag}_pytest.log
for f in bench_1 rn_b512_1 rn_b256_1 bert_1 tuner_1; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log | tail -1) $(grep -o '"run_to_first_step_s": [0-9.]*' gpurun_out/${tag}_$f.log | tail -1)"; done
tail -2 gpurun_out/${tag}_smoke.log
echo SESSION_DONE
