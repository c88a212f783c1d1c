#!/usr/bin/env bash
# Round-5 session 3: stream-K GEMM (numerics, isolated A/B on BERT shapes, BERT end to end).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s3}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 240 ${tag}_gb.log bin/gemm_bench 20 8192,2304,768,0 8192,3072,768,0 8192,768,3072,0 8192,768,768,0 8192,768,2304,1 8192,3072,768,1 8192,768,3072,1 4096,4096,4096,0 8192,8192,8192,0 || exit 1
$S 300 ${tag}_sk.log python -u -m pytest tests/test_gemm_streamk_gpu.py tests/test_gemm256_gpu.py -x -v --timeout 120 --timeout-method thread || exit 1
chk ${tag}_sk.log
$S 300 ${tag}_bt.log python -u -m pytest tests/test_bert_hf_parity.py tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_bt.log
for r in 1 2; do
CLOUD_AMD_GEMM_STREAMK=0 $S 200 ${tag}_bert_sk0_${r}.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_GEMM_STREAMK=1 $S 200 ${tag}_bert_sk1_${r}.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
done
grep -h '"variant"' gpurun_out/${tag}_gb.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('%-9s %5d %5d %5d L%d %8.1f us %7.1f TF bad=%d' % (d['variant'],d['M'],d['N'],d['K'],d['layout'],d['us'],d['TF'],d['bad']))"
tail -2 gpurun_out/${tag}_sk.log
for f in gpurun_out/${tag}_bert_sk*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
