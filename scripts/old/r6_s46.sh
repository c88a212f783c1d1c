#!/usr/bin/env bash
# Round-6 session 46: remaining ResNet-50 knobs re-checked on the final tree, interleaved:
# stem weight-gradient split target, BN finalize group rows, host run-ahead depth.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s46
for r in 1 2; do
$S 200 ${tag}_rn_def_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_STEM_WGRAD_BLOCKS=1024 $S 200 ${tag}_rn_stem1024_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_STEM_WGRAD_BLOCKS=4096 $S 200 ${tag}_rn_stem4096_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FIN_RPG=256 $S 200 ${tag}_rn_rpg256_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_MAX_STEPS_IN_FLIGHT=3 $S 200 ${tag}_rn_depth3_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
