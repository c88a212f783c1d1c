#!/usr/bin/env bash
# A/B: weight-gradient GEMMs on a side stream in the ResNet block backward.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
$S 300 bench_ws0.log env CLOUD_AMD_WGRAD_STREAM=0 python bench.py --steps 30 --warmup 5 || exit 1
$S 300 bench_ws1.log python bench.py --steps 30 --warmup 5 || exit 1
$S 300 bench_ws1_graph.log python bench.py --steps 30 --warmup 5 --graph 1 || exit 1
$S 300 bench_ws0b.log env CLOUD_AMD_WGRAD_STREAM=0 python bench.py --steps 30 --warmup 5 || exit 1
$S 300 bench_ws1b.log python bench.py --steps 30 --warmup 5 || exit 1
echo SESSION_DONE
