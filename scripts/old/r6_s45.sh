#!/usr/bin/env bash
# Round-6 session 45: weight-gradient split-K targets on the final tree (CLOUD_AMD_WGRAD_BLOCKS /
# _SMALLM 512 default vs 384 / 768), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s45
for r in 1 2; do
$S 200 ${tag}_rn_512_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_WGRAD_BLOCKS=384 CLOUD_AMD_WGRAD_BLOCKS_SMALLM=384 $S 200 ${tag}_rn_384_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_WGRAD_BLOCKS=768 CLOUD_AMD_WGRAD_BLOCKS_SMALLM=768 $S 200 ${tag}_rn_768_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
