#!/usr/bin/env bash
# Round-6 session 30: adaptive step-pacer depth (CLOUD_AMD_RUN_AHEAD_MS) -- pacer tests, BERT A/B
# interleaved (0 = fixed depth 2 vs default 25 ms), one ResNet run (depth must stay 2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s30
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 300 ${tag}_pt.log python -u -m pytest tests/test_step_pacer_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_pt.log
tail -1 gpurun_out/${tag}_pt.log
for r in 1 2 3; do
CLOUD_AMD_RUN_AHEAD_MS=0 $S 200 ${tag}_bert_fixed_$r.log python bench/bert_base_synth.py --steps 40 --warmup 6 || exit 1
$S 200 ${tag}_bert_adapt_$r.log python bench/bert_base_synth.py --steps 40 --warmup 6 || exit 1
done
$S 200 ${tag}_rn.log python bench.py --steps 20 --warmup 5 || exit 1
for f in gpurun_out/${tag}_bert_*.log gpurun_out/${tag}_rn.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1) $(grep -o '"max_steps_in_flight": [0-9a-z]*' $f | tail -1) $(grep -o '"pacer_step_ms": [0-9.a-z]*' $f | tail -1) $(grep -o '"unpaced_median_ms": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
