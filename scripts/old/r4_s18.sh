#!/usr/bin/env bash
# Round-4 session 18: 256 x 128 single-phase GEMM core -- numerics (library tests + standalone
# bench vs fp32), BERT-shape timings, BERT A/B (CLOUD_AMD_GEMM_256X128=1 default vs 0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s18}
out=gpurun_out/$tag; mkdir -p $out
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 300 ${tag}_g256_tests.log python -u -m pytest tests/test_gemm256_gpu.py tests/test_plain_gemm_policy_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_g256_tests.log
timeout -k 10 240 bin/gemm_bench 20 8192,3072,768,0 8192,3072,768,1 8192,2304,768,0 4096,4096,4096,0 8192,8192,8192,0 8000,1000,704,0 > $out/gemm_bench.txt 2>&1 || { echo "gemm_bench failed"; cat $out/gemm_bench.txt; exit 1; }
grep -h '"variant"' $out/gemm_bench.txt | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['variant'],d['M'],d['N'],d['K'],d['layout'],d['TF'],d['bad'])"
for i in 1 2; do
$S 240 ${tag}_bert_${i}.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_GEMM_256X128=0 $S 240 ${tag}_bert_off_${i}.log python bench/bert_base_synth.py || exit 1
done
$S 240 ${tag}_rn.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
for f in bert_1 bert_off_1 bert_2 bert_off_2 rn; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log | tail -1)"; done
echo SESSION_DONE
