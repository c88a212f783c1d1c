#!/usr/bin/env bash
# Round-6 session 22: weight-gradient side stream on a CU-masked stream (1/2, 1/4 of the CUs)
# vs all CUs, BERT x2 / ResNet x2 per arm, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s22
for r in 1 2; do
for f in 0 0.5 0.25 0.375; do
CLOUD_AMD_SIDE_CU_FRAC=$f $S 200 ${tag}_bert_f${f}_$r.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
done
done
for r in 1 2; do
for f in 0 0.5 0.25; do
CLOUD_AMD_SIDE_CU_FRAC=$f $S 200 ${tag}_rn_f${f}_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
done
for f in gpurun_out/${tag}_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
