#!/usr/bin/env bash
# Round-5 session 31: software-pipelined LayerNorm forward (CLOUD_AMD_LN_FWD_PF, grid
# CLOUD_AMD_LN_FWD_BLOCKS): transformer GPU tests with it on, BERT interleaved off / 512 / 1024.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s31}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
CLOUD_AMD_LN_FWD_PF=1 $S 300 ${tag}_t.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py tests/test_keras_native_gpu.py || exit 1
chk ${tag}_t.log
tail -1 gpurun_out/${tag}_t.log
run() { local name=$1; shift; env "$@" timeout -k 10 200 python bench/bert_base_synth.py --steps 20 --warmup 5 > gpurun_out/${tag}_${name}.log 2>&1 || { echo "fail $name"; exit 1; }; echo "$name $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_${name}.log | tail -1)"; }
for i in 1 2 3; do
run off_$i CLOUD_AMD_LN_FWD_PF=0
run pf512_$i CLOUD_AMD_LN_FWD_PF=1 CLOUD_AMD_LN_FWD_BLOCKS=512
run pf1024_$i CLOUD_AMD_LN_FWD_PF=1 CLOUD_AMD_LN_FWD_BLOCKS=1024
done
rm -rf gpurun_out/${tag}_bprof
CLOUD_AMD_LN_FWD_PF=1 CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_bprof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_bprof -o run --output-format csv -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_bprof adam_kernel > gpurun_out/${tag}_bert_step_kernels.txt || true
rm -rf gpurun_out/${tag}_bprof
grep -E "ln_fwd|kernel time" gpurun_out/${tag}_bert_step_kernels.txt | head -4
echo SESSION_DONE
