#!/usr/bin/env bash
# Round-5 session 20: BERT knob sweep on the current tree (dense weight-gradient split target,
# prefetching dense epilogue), interleaved, two runs each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s20}
for r in 1 2; do
for b in 640 256 384 1024; do
CLOUD_AMD_DENSE_WGRAD_BLOCKS=$b $S 200 ${tag}_b${b}_$r.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
done
CLOUD_AMD_EPI_PF=0 $S 200 ${tag}_pf0_$r.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
