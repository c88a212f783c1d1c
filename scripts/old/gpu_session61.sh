#!/usr/bin/env bash
# BERT-base: 2-rank DP rehearsal on one GPU (gloo, shared device) and a current kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
CLOUD_AMD_SHARED_GPU=1 CLOUD_AMD_DIST_BACKEND=gloo $S 240 bert_dp2_rehearsal.log \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 \
  bench/bert_base_synth.py --gpus 2 --steps 5 --warmup 3 || exit 1
$S 300 prof_bert.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o run -- python bench/bert_base_synth.py --steps 10 --warmup 3 || exit 1
echo SESSION_DONE
