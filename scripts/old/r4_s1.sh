#!/usr/bin/env bash
# Round-4 session 1: the RCCL data-plane tests (world-1 nccl group, reducer forced to
# world 2, torch.distributed and native RcclComm, bf16/fp32 wire), the mid-backward
# failure test, then smoke + full GPU suite + ResNet-50 / BERT benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s1}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 400 ${tag}_new.log python -u -m pytest tests/test_rccl_dataplane_gpu.py tests/test_transformer_gpu.py -k "dataplane or rccl or raising" -x -v --timeout 120 --timeout-method thread || exit 1
chk ${tag}_new.log
$S 300 ${tag}_smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S 900 ${tag}_pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_pytest.log
$S 240 ${tag}_bench_1.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 240 ${tag}_bert_1.log python bench/bert_base_synth.py || exit 1
tail -1 gpurun_out/${tag}_pytest.log
for f in bench_1 bert_1; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log | tail -1)"; done
echo SESSION_DONE
