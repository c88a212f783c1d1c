#!/usr/bin/env bash
# Headline via run(): stage + launch one rank through cloud_amd.run(); BERT kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 400 via_run.log python bench.py --via-run 1 --steps 20 --warmup 5 || exit 1
$S 300 prof_bert.log env CLOUD_AMD_WGRAD_STREAM=0 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert2 -o run -- python bench/bert_base_synth.py --steps 10 --warmup 3 || exit 1
echo SESSION_DONE
