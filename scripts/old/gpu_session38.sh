#!/usr/bin/env bash
# Re-verify after the revert; BERT with the 8-wave double-buffered core (A/B).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "FAILED\|ERROR" gpurun_out/pytest_gpu.log && { echo "gpu tests failed"; exit 1; }
$S 300 bench.log python bench.py --steps 20 --warmup 5 || exit 1
$S 300 bert_g4.log python bench/bert_base_synth.py --steps 40 --warmup 8 || exit 1
$S 300 bert_g8.log env CLOUD_AMD_GEMM_CORE=glds8 python bench/bert_base_synth.py --steps 40 --warmup 8 || exit 1
$S 300 bert_g4b.log python bench/bert_base_synth.py --steps 40 --warmup 8 || exit 1
$S 300 bert_g8b.log env CLOUD_AMD_GEMM_CORE=glds8 python bench/bert_base_synth.py --steps 40 --warmup 8 || exit 1
echo SESSION_DONE
