#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 ab_glds.log env CLOUD_AMD_GEMM_CORE=glds python bench/gemm_core_ab.py || exit 1
$S 300 ab_reg.log env CLOUD_AMD_GEMM_CORE=reg python bench/gemm_core_ab.py || exit 1
$S 600 pytest_gpu.log python -m pytest tests -m gpu -q || exit 1
$S 400 bench_bert.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
$S 400 bench_native.log python bench.py --steps 20 --warmup 5 || exit 1
$S 400 bench_via_run.log python bench.py --via-run 1 --steps 10 --warmup 3 || exit 1
echo SESSION_DONE
