#!/usr/bin/env bash
# M=64 weight-gradient tile / pipeline variants (env switch WGRAD64 of the reverted experiment, conv.hip) x split-K targets, then end-to-end.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
for v in 0 1 2 3; do
  WGRAD64=$v $S 200 r2s25_sweep_v$v.log python bench/wgrad_sweep.py 1024 256,512,1024,2048 || exit 1
done
for i in 1 2; do
  for v in 0 1 2 3; do
    WGRAD64=$v $S 200 r2s25_bench_v${v}_$i.log python bench.py --via-run 0 || exit 1
  done
done
echo SESSION_DONE
