#!/usr/bin/env bash
# Round-3 session 23: the driver's round-end checks on the final tree (smoke, full GPU suite,
# bench command), 2-rank DP rehearsals of both benches on one GPU over gloo, tuner with the
# early footprint report, BERT repeats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s23}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 300 ${tag}_smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S 900 ${tag}_pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_pytest.log
$S 240 ${tag}_bench.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_SHARED_GPU=1 CLOUD_AMD_DIST_BACKEND=gloo CLOUD_AMD_NUM_GPUS=2 $S 300 ${tag}_dp2_resnet.log python bench.py --gpus 2 --steps 4 --warmup 2 --batch 128 || exit 1
CLOUD_AMD_SHARED_GPU=1 CLOUD_AMD_DIST_BACKEND=gloo CLOUD_AMD_NUM_GPUS=2 $S 300 ${tag}_dp2_bert.log python bench/bert_base_synth.py --gpus 2 --steps 4 --warmup 2 || exit 1
for i in 1 2; do
$S 400 ${tag}_tuner_${i}.log python bench/tuner_8trials.py || exit 1
$S 240 ${tag}_bert_${i}.log python bench/bert_base_synth.py || exit 1
done
grep -h '"metric"' gpurun_out/${tag}_dp2_resnet.log gpurun_out/${tag}_dp2_bert.log | cut -c1-600
for f in bench tuner_1 bert_1 tuner_2 bert_2; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log)"; done
tail -2 gpurun_out/${tag}_smoke.log
echo SESSION_DONE
