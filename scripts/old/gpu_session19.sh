#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 ddp_event.log python scripts/ddp_probe.py || exit 1
$S 300 pytest_ddp_gpu.log python -m pytest tests/test_ddp_gpu.py -q || exit 1
$S 600 pytest_gpu.log python -m pytest tests -m gpu -q || exit 1
$S 400 bench.log python bench.py --steps 20 --warmup 5 || exit 1
$S 400 bench_bert.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
$S 300 graph.log python bench.py --graph 1 --steps 10 --warmup 3 || exit 1
echo SESSION_DONE
