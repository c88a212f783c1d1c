#!/usr/bin/env bash
# Round-6 session 25: world-2 shared-GPU rehearsals (gloo) of both benches with the DP A/B cells.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s25
export CLOUD_AMD_JOBS_DIR=$PWD/gpurun_out/${tag}_jobs
export CLOUD_AMD_SHARED_GPU=1 CLOUD_AMD_DIST_BACKEND=gloo CLOUD_AMD_NUM_GPUS=2
$S 400 ${tag}_rn_dp2.log python bench.py --gpus 2 --steps 5 --warmup 3 --batch 128 || exit 1
$S 400 ${tag}_bert_dp2.log python bench/bert_base_synth.py --gpus 2 --steps 5 --warmup 3 || exit 1
rm -rf gpurun_out/${tag}_jobs
for f in gpurun_out/${tag}_*dp2.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1) $(grep -o '"replicas_consistent": [a-z]*' $f | tail -1) cells=$(grep -o '"exposed_comm_ms"' $f | wc -l)"; done
echo SESSION_DONE
