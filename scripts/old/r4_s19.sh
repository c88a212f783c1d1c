#!/usr/bin/env bash
# Round-4 session 19: the driver's round-end checks on the current tree (smoke, full GPU suite,
# bench command twice), BERT, the tuner bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s19}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 300 ${tag}_smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S 900 ${tag}_pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_pytest.log
for i in 1 2; do
$S 240 ${tag}_bench_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
done
$S 240 ${tag}_bert.log python bench/bert_base_synth.py || exit 1
$S 300 ${tag}_tuner.log python bench/tuner_8trials.py || exit 1
tail -1 gpurun_out/${tag}_pytest.log
for f in bench_1 bench_2 bert tuner; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log | tail -1)"; done
echo SESSION_DONE
