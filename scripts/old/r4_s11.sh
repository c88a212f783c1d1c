#!/usr/bin/env bash
# Round-4 session 11: two-phase 256 core as the default large-GEMM core -- full GPU suite, then
# default vs the ring core (CLOUD_AMD_GEMM_CORE=glds_ring) on the GEMM A/B, ResNet-50 and BERT.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s11}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 600 ${tag}_pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_pytest.log
$S 300 ${tag}_gemm_p8.log python bench/gemm_core_ab.py || exit 1
CLOUD_AMD_GEMM_CORE=glds_ring $S 300 ${tag}_gemm_ring.log python bench/gemm_core_ab.py || exit 1
for i in 1 2; do
$S 240 ${tag}_rn_p8_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_GEMM_CORE=glds_ring $S 240 ${tag}_rn_ring_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 240 ${tag}_bert_p8_${i}.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_GEMM_CORE=glds_ring $S 240 ${tag}_bert_ring_${i}.log python bench/bert_base_synth.py || exit 1
done
tail -1 gpurun_out/${tag}_pytest.log
grep -h summary gpurun_out/${tag}_gemm_*.log
for f in rn_p8_1 rn_ring_1 rn_p8_2 rn_ring_2 bert_p8_1 bert_ring_1 bert_p8_2 bert_ring_2; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log | tail -1)"; done
echo SESSION_DONE
