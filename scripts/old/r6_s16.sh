#!/usr/bin/env bash
# Round-6 session 16: single-threaded vs multithreaded autograd backward, interleaved A/B
# (BERT x3 each, ResNet x2 each), host launch time in the JSON.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s16
for r in 1 2 3; do
$S 200 ${tag}_bert_st_$r.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_AUTOGRAD_MT=1 $S 200 ${tag}_bert_mt_$r.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
done
for r in 1 2; do
$S 200 ${tag}_rn_st_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_AUTOGRAD_MT=1 $S 200 ${tag}_rn_mt_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1) $(grep -o '"unpaced_median_ms": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
