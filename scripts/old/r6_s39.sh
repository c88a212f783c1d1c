#!/usr/bin/env bash
# Round-6 session 39: every BN fold site (CLOUD_AMD_BN_FOLD_ALL=1) on the final tree, where the
# N % 256 sites now run on the two-deep tiles; and stage 4 (MAX_N=512) again, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s39
for r in 1 2; do
$S 200 ${tag}_rn_def_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD_ALL=1 $S 200 ${tag}_rn_all_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD_MAX_N=512 $S 200 ${tag}_rn_n512_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
