#!/usr/bin/env bash
# Round-5 session 17: packed-FP32 GELU / GELU' dense epilogues: numerics (dense + BERT parity
# tests), epilogue costs, BERT bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s17}
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
$S 400 ${tag}_t.log $PT tests/test_bert_hf_parity.py tests/test_gemm_streamk_gpu.py tests/test_gemm_256x96_gpu.py tests/test_kernels_gpu.py -k "gelu or bert or dense or gemm or 256x96 or streamk" || exit 1
grep -q "FAILED\|Error" gpurun_out/${tag}_t.log && { echo T_FAILED; tail -40 gpurun_out/${tag}_t.log; exit 1; }
grep -E "passed|failed" gpurun_out/${tag}_t.log | tail -1
$S 200 ${tag}_epi.log python bench/dense_epilogue_cost.py || exit 1
grep case gpurun_out/${tag}_epi.log
for r in 1 2; do
$S 200 ${tag}_bert_$r.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
done
for r in 1 2; do
$S 200 ${tag}_rn_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_bert_*.log gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
