#!/usr/bin/env bash
# Round-3 session 6: embedding / LayerNorm backward latency fixes -- transformer tests, BERT bench + profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s6}
$S 400 ${tag}_pytest.log python -u -m pytest tests/test_transformer_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/${tag}_pytest.log && ! grep -qE " failed| error" gpurun_out/${tag}_pytest.log || { echo "GPU tests failed"; tail -40 gpurun_out/${tag}_pytest.log; exit 1; }
$S 240 ${tag}_bert.log python bench/bert_base_synth.py || exit 1
scripts/r3_prof_bert.sh ${tag} || exit 1
grep -o '"value": [0-9.]*' gpurun_out/${tag}_bert.log
echo SESSION_DONE
