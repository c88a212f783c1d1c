#!/usr/bin/env bash
# Round-5 session 6: 128 x 192 tiles on BERT forward shapes (isolated A/B); the stock row with
# MIOpen find (torch.backends.cudnn.benchmark = True) next to cloud_amd via run(), same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s6}
GB_VARIANTS=glds128,g128x192,p8h2 $S 200 ${tag}_gb.log bin/gemm_bench 20 8192,2304,768,0 8192,3072,768,0 8192,768,3072,0 8192,768,768,0 4096,4096,4096,0 || exit 1
grep -h '"variant"' gpurun_out/${tag}_gb.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('%-9s %5d %5d %5d L%d %8.1f us %7.1f TF bad=%d rel=%.2e' % (d['variant'],d['M'],d['N'],d['K'],d['layout'],d['us'],d['TF'],d['bad'],d['rel_l2']))"
$S 200 ${tag}_rn.log python bench.py --steps 20 --warmup 5 || exit 1
$S 900 ${tag}_stock_bm1.log python bench/stock_resnet50.py --benchmark 1 --steps 20 --warmup 5 || exit 1
for f in gpurun_out/${tag}_rn.log gpurun_out/${tag}_stock_bm1.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1) $(grep -o '"first_step_latency_s": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
