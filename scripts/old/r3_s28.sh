#!/usr/bin/env bash
# Round-3 session 28: tuner standbys with the HIP context + kernel library created before the
# gate (A/B against CLOUD_AMD_TUNER_STANDBY_HIP=0, interleaved), timelines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s28}
for i in 1 2 3; do
$S 300 ${tag}_tuner_hip1_${i}.log python bench/tuner_8trials.py || exit 1
CLOUD_AMD_TUNER_STANDBY_HIP=0 $S 300 ${tag}_tuner_hip0_${i}.log python bench/tuner_8trials.py || exit 1
done
for a in hip1 hip0; do for i in 1 2 3; do grep -h '"metric"' gpurun_out/${tag}_tuner_${a}_${i}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a', d['value'], d['wall_s'], d['trials_completed'])"; done; done
grep -h '"metric"' gpurun_out/${tag}_tuner_hip1_1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); [print(k, v) for k, v in d['timeline']['workers'].items()]; [print(t) for t in d['timeline']['trials']]"
echo SESSION_DONE
