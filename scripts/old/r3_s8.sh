#!/usr/bin/env bash
# Round-3 session 8: batched gradient finalisation -- transformer tests, BERT bench A/B + profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s8}
$S 400 ${tag}_pytest.log python -u -m pytest tests/test_transformer_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/${tag}_pytest.log && ! grep -qE " failed| error" gpurun_out/${tag}_pytest.log || { echo "GPU tests failed"; tail -40 gpurun_out/${tag}_pytest.log; exit 1; }
$S 240 ${tag}_bert.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_GRAD_FIN_BATCH=0 $S 240 ${tag}_bert_f0.log python bench/bert_base_synth.py || exit 1
$S 240 ${tag}_bert2.log python bench/bert_base_synth.py || exit 1
scripts/r3_prof_bert.sh ${tag} || exit 1
for f in bert bert_f0 bert2; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log)"; done
echo SESSION_DONE
