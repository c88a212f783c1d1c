#!/usr/bin/env bash
# Re-verify the rebuilt tree after the container re-creation: gpu tests, smoke, benches, rocprof.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 600 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
$S 300 smoke.log python __graft_entry__.py smoke || exit 1
$S 400 bench.log python bench.py --steps 20 --warmup 5 || exit 1
$S 400 bench_bert.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
$S 400 prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_resnet -o run -- python bench.py --steps 10 --warmup 3 || exit 1
echo SESSION_DONE
