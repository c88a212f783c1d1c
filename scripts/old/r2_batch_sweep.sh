#!/usr/bin/env bash
# ResNet-50 per-GPU batch sweep on one box (in-process ranks, same binary).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
for b in 512 768 1024 1536 2048; do
  $S 300 sweep_b$b.log python bench.py --via-run 0 --batch $b --steps 10 --warmup 5 || exit 1
done
echo SESSION_DONE
