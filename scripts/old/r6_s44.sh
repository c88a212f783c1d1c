#!/usr/bin/env bash
# Round-6 session 44: last tree check -- full GPU suite + smoke, ResNet-50 x2, BERT x1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${TAG:-r6s44}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 1000 ${tag}_all.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs || exit 1
chk ${tag}_all.log
tail -2 gpurun_out/${tag}_all.log
$S 300 ${tag}_smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" || exit 1
tail -1 gpurun_out/${tag}_smoke.log
for r in 1 2; do
$S 200 ${tag}_rn_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
$S 200 ${tag}_bert_1.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
for f in gpurun_out/${tag}_rn_*.log gpurun_out/${tag}_bert_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
