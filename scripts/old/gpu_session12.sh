#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 600 pytest_gpu.log python -m pytest tests -m gpu -q -x || exit 1
$S 300 conv_shapes.log python bench/conv_shapes.py || exit 1
$S 400 bench_native.log python bench.py --steps 20 --warmup 5 || exit 1
$S 400 bench_bert.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
$S 500 prof_native.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_native -o run --output-format csv -- python bench.py --steps 5 --warmup 3 || exit 1
echo SESSION_DONE
