#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 pytest_ddp_gpu.log python -m pytest tests/test_ddp_gpu.py -q -x || exit 1
$S 600 pytest_gpu.log python -m pytest tests -m gpu -q || exit 1
$S 500 prof_bert.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o run --output-format csv -- python bench/bert_base_synth.py --steps 5 --warmup 3 || exit 1
$S 300 graph.log python bench.py --graph 1 --steps 10 --warmup 3 || exit 1
echo SESSION_DONE
