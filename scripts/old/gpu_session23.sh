#!/usr/bin/env bash
# Per-GPU batch sweep (ours) + stock comparator at 256 / 512.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 bench_b384.log python bench.py --steps 20 --warmup 5 --batch 384 || exit 1
$S 300 bench_b512.log python bench.py --steps 20 --warmup 5 --batch 512 || exit 1
$S 300 bench_b768.log python bench.py --steps 15 --warmup 5 --batch 768 || exit 1
$S 300 bench_b1024.log python bench.py --steps 10 --warmup 4 --batch 1024 || exit 1
$S 400 stock_b256.log python bench/stock_resnet50.py --steps 20 --warmup 5 --batch 256 || exit 1
$S 400 stock_b512.log python bench/stock_resnet50.py --steps 20 --warmup 5 --batch 512 || exit 1
echo SESSION_DONE
