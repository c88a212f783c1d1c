#!/usr/bin/env bash
# Round-6 session 20: 8-wave two-stage 128 x 64 dense GEMMs -- full GPU suite, BERT A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s20
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 1000 ${tag}_all.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
chk ${tag}_all.log
tail -2 gpurun_out/${tag}_all.log
for r in 1 2 3; do
$S 200 ${tag}_bert_on_$r.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_GEMM_W8N64=0 $S 200 ${tag}_bert_off_$r.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
done
$S 200 ${tag}_rn_1.log python bench.py --steps 20 --warmup 5 || exit 1
for f in gpurun_out/${tag}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
