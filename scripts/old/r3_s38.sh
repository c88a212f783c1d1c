#!/usr/bin/env bash
# Round-3 session 38: the reference's multi-process Keras workloads through run() with two
# ranks sharing the one GPU over gloo (the DP path on device tensors): the custom training
# loop (chief + worker, MultiWorkerMirrored) and run() inside a script (Keras fit, Mirrored).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s38}
export CLOUD_AMD_SHARED_GPU=1 CLOUD_AMD_DIST_BACKEND=gloo CLOUD_AMD_NUM_GPUS=2 CLOUD_AMD_EXAMPLE_SMALL=1
export CLOUD_AMD_JOBS_DIR=$PWD/gpurun_out/${tag}_jobs
$S 300 ${tag}_ctl.log python examples/call_run_on_script_with_keras_ctl.py || exit 1
$S 400 ${tag}_within.log python examples/call_run_within_script_with_keras_fit.py || exit 1
grep -h "RESULT" gpurun_out/${tag}_jobs/*/logs/*.log | head -8
tail -3 gpurun_out/${tag}_ctl.log gpurun_out/${tag}_within.log
echo SESSION_DONE
