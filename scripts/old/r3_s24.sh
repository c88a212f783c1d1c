#!/usr/bin/env bash
# Round-3 session 24: dense weight-gradient engine microbench (in-tree split-K vs hipBLASLt
# bf16->fp32), tuner runs with the per-worker timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s24}
$S 200 ${tag}_wgrad_lib.log python bench/wgrad_lib.py || exit 1
for i in 1 2; do
$S 300 ${tag}_tuner_${i}.log python bench/tuner_8trials.py || exit 1
done
grep -v amdgpu.ids gpurun_out/${tag}_wgrad_lib.log
for i in 1 2; do grep -h '"metric"' gpurun_out/${tag}_tuner_${i}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['wall_s']); [print(k, v) for k, v in d['timeline']['workers'].items()]; [print(t) for t in d['timeline']['trials']]"; done
echo SESSION_DONE
