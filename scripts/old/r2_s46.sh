#!/usr/bin/env bash
# Critical path on a high-priority stream (reverted MAIN_PRIORITY switch in bench.py) vs default, ResNet-50 b1024.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
for i in 1 2 3; do
  MAIN_PRIORITY=0 $S 200 r2s46_p0_$i.log python bench.py --via-run 0 || exit 1
  MAIN_PRIORITY=1 $S 200 r2s46_p1_$i.log python bench.py --via-run 0 || exit 1
done
echo SESSION_DONE
