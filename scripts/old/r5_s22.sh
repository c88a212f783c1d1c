#!/usr/bin/env bash
# Round-5 session 22: per-bucket optimizer at world 1 (AdamW / SGD slices beside backward):
# bitwise test vs the whole-arena step, RCCL data-plane tests, BERT / ResNet-50 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s22}
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
$S 600 ${tag}_t.log $PT tests/test_sliced_opt_world1_gpu.py tests/test_rccl_dataplane_gpu.py tests/test_ctl_gpu.py || exit 1
grep -q "FAILED\|Error" gpurun_out/${tag}_t.log && { echo T_FAILED; tail -40 gpurun_out/${tag}_t.log; exit 1; }
grep -E "passed|failed" gpurun_out/${tag}_t.log | tail -1
for r in 1 2 3; do
$S 200 ${tag}_bert_s1_$r.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_SLICED_OPT=0 $S 200 ${tag}_bert_s0_$r.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
$S 200 ${tag}_rn_s1_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_SLICED_OPT=0 $S 200 ${tag}_rn_s0_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_bert_*.log gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1) $(grep -o '"sliced_optimizer": [a-z]*' $f | tail -1)"; done
echo SESSION_DONE
