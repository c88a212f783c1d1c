#!/usr/bin/env bash
# Final verification of the tree: all GPU tests, smoke, headline bench, graph path, BERT, via run().
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
grep -q "FAILED\|ERROR" gpurun_out/pytest_gpu.log && { echo "gpu tests failed"; exit 1; }
$S 300 smoke.log python __graft_entry__.py smoke || exit 1
$S 300 bench.log python bench.py || exit 1
$S 300 bench_graph.log python bench.py --graph 1 --steps 10 --warmup 3 || exit 1
$S 300 bert.log python bench/bert_base_synth.py --steps 40 --warmup 8 || exit 1
$S 400 via_run.log python bench.py --via-run 1 --steps 20 --warmup 5 || exit 1
echo SESSION_DONE
