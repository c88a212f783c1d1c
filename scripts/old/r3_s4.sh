#!/usr/bin/env bash
# Round-3 session 4: fused short-sequence attention + in-launch split-K -- full GPU suite,
# smoke, BERT and ResNet benches, BERT per-step kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s4}
$S 700 ${tag}_pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/${tag}_pytest.log && ! grep -qE " failed| error" gpurun_out/${tag}_pytest.log || { echo "GPU tests failed"; tail -40 gpurun_out/${tag}_pytest.log; exit 1; }
$S 200 ${tag}_smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S 240 ${tag}_bert.log python bench/bert_base_synth.py || exit 1
$S 240 ${tag}_bench.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
scripts/r3_prof_bert.sh ${tag} || exit 1
echo SESSION_DONE
