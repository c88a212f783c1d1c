#!/usr/bin/env bash
# Round-6 session 15: host launch path (single-threaded backward, raw stream handles, native
# side-stream fork) -- full GPU suite, host profile, BERT x3, ResNet x2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s15
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 1000 ${tag}_all.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
chk ${tag}_all.log
tail -2 gpurun_out/${tag}_all.log
$S 300 ${tag}_host.txt python -u scripts/host_profile.py bert 20 || exit 1
head -3 gpurun_out/${tag}_host.txt
for r in 1 2 3; do
$S 200 ${tag}_bert_$r.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
done
for r in 1 2; do
$S 200 ${tag}_rn_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_rn_*.log gpurun_out/${tag}_bert_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1) $(grep -o '"unpaced_median_ms": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
