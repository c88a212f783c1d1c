#!/usr/bin/env bash
# Round-3 session 5: in-launch split-K (sc1 slabs) A/B on BERT and ResNet, + BERT profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s5}
$S 400 ${tag}_pytest.log python -u -m pytest tests/test_transformer_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/${tag}_pytest.log && ! grep -qE " failed| error" gpurun_out/${tag}_pytest.log || { echo "GPU tests failed"; tail -40 gpurun_out/${tag}_pytest.log; exit 1; }
$S 240 ${tag}_bert.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_SPLITK_INLAUNCH=0 $S 240 ${tag}_bert_sep.log python bench/bert_base_synth.py || exit 1
$S 240 ${tag}_bench.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_SPLITK_INLAUNCH=0 $S 240 ${tag}_bench_sep.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
scripts/r3_prof_bert.sh ${tag} || exit 1
for f in bert bert_sep bench bench_sep; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log)"; done
echo SESSION_DONE
