#!/usr/bin/env bash
# Multi-rank rehearsal of the driver's N=2 bench path on a one-GPU box: bench.py under
# torch.distributed.run with 2 ranks, both on cuda:0, gloo transport (RCCL refuses two
# ranks on one device). Checks the barrier/max-over-ranks timing, parameter broadcast,
# bucketed all-reduce and the single rank-0 JSON line. Then BERT-base bench for current numbers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
CLOUD_AMD_SHARED_GPU=1 CLOUD_AMD_DIST_BACKEND=gloo $S 240 bench_dp2_rehearsal.log \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus 2 --steps 5 --warmup 3 --batch 128 || exit 1
grep -c '"metric"' gpurun_out/bench_dp2_rehearsal.log
$S 300 bench_bert.log python bench/bert_base_synth.py || exit 1
echo SESSION_DONE
