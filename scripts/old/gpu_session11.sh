#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 600 pytest_gpu.log python -m pytest tests -m gpu -q -x || exit 1
$S 300 conv_shapes.log python bench/conv_shapes.py || exit 1
$S 300 ab_glds.log python bench/gemm_core_ab.py || exit 1
$S 400 bench_native.log python bench.py --steps 20 --warmup 5 || exit 1
$S 400 bench_bert.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
echo SESSION_DONE
