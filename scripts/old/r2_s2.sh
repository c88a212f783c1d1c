#!/usr/bin/env bash
# Round 2 session 2: KFD topology dump, bench via run() (default), BERT via run(), 2-rank shared-GPU rehearsal.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
mkdir -p gpurun_out/kfd
for n in /sys/class/kfd/kfd/topology/nodes/*; do
  b=$(basename $n); mkdir -p gpurun_out/kfd/$b
  cp $n/properties gpurun_out/kfd/$b/ 2>/dev/null
  for sub in mem_banks io_links; do
    for d in $n/$sub/*; do [ -e "$d/properties" ] && mkdir -p gpurun_out/kfd/$b/$sub/$(basename $d) && cp $d/properties gpurun_out/kfd/$b/$sub/$(basename $d)/; done
  done
done
python -c "import json; from cloud_amd.core import topology as t; print(json.dumps(t.describe_node()))" > gpurun_out/r2s2_node.json 2>&1
$S 300 r2s2_bench_via_run.log python bench.py || exit 1
$S 300 r2s2_bert_via_run.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_SHARED_GPU=1 CLOUD_AMD_DIST_BACKEND=gloo CLOUD_AMD_NUM_GPUS=2 $S 300 r2s2_dp2_rehearsal.log python bench.py --gpus 2 --steps 4 --warmup 2 --batch 128 || exit 1
echo SESSION_DONE
