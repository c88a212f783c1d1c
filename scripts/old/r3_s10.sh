#!/usr/bin/env bash
# Round-3 session 10: two-blocks-per-CU fused attention backward; dense wgrad split-K
# block target A/B (1024 default vs 512 / 768); BERT profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s10}
$S 400 ${tag}_pytest.log python -u -m pytest tests/test_transformer_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/${tag}_pytest.log && ! grep -qE " failed| error" gpurun_out/${tag}_pytest.log || { echo "GPU tests failed"; tail -40 gpurun_out/${tag}_pytest.log; exit 1; }
$S 240 ${tag}_bert.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_DENSE_WGRAD_BLOCKS=512 $S 240 ${tag}_bert_w512.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_DENSE_WGRAD_BLOCKS=768 $S 240 ${tag}_bert_w768.log python bench/bert_base_synth.py || exit 1
$S 240 ${tag}_bert2.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_DENSE_WGRAD_BLOCKS=512 $S 240 ${tag}_bert_w512b.log python bench/bert_base_synth.py || exit 1
scripts/r3_prof_bert.sh ${tag} || exit 1
for f in bert bert_w512 bert_w768 bert2 bert_w512b; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log)"; done
echo SESSION_DONE
