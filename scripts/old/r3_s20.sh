#!/usr/bin/env bash
# Round-3 session 20: attention forward with P staged in the dead K image (36 KB LDS, three
# blocks per CU): transformer / HF parity tests, BERT bench, BERT per-step kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s20}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 300 ${tag}_t1.log python -u -m pytest tests/test_transformer_gpu.py tests/test_bert_hf_parity.py -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_t1.log
for i in 1 2; do
$S 240 ${tag}_bert_${i}.log python bench/bert_base_synth.py || exit 1
done
rm -rf gpurun_out/${tag}_prof_bert
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_prof_bert.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_bert -o run --output-format csv -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof_bert adam_kernel > gpurun_out/${tag}_bert_step_kernels.txt
rm -rf gpurun_out/${tag}_prof_bert
head -20 gpurun_out/${tag}_bert_step_kernels.txt
for f in bert_1 bert_2; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log)"; done
echo SESSION_DONE
