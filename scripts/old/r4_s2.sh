#!/usr/bin/env bash
# Round-4 session 2: BN-fold kernels (ca_gemm_xa.h) vs fp32 + bitwise vs the unfused path,
# RCCL data-plane tests, ResNet-50 fold A/B, serialized step profile, full GPU suite, BERT.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s2}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 400 ${tag}_new.log python -u -m pytest tests/test_bn_fold_gpu.py tests/test_rccl_dataplane_gpu.py tests/test_transformer_gpu.py -k "fold or bnbwd or dataplane or rccl or raising" -x -v --timeout 120 --timeout-method thread || exit 1
chk ${tag}_new.log
for i in 1 2; do
CLOUD_AMD_BN_FOLD=0 $S 240 ${tag}_rn_off_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD=1 $S 240 ${tag}_rn_on_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
done
rm -rf gpurun_out/${tag}_prof_rn
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_prof_rn.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_rn -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof_rn sgd_kernel > gpurun_out/${tag}_rn_step_kernels.txt
rm -rf gpurun_out/${tag}_prof_rn
head -30 gpurun_out/${tag}_rn_step_kernels.txt
$S 900 ${tag}_pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_pytest.log
$S 240 ${tag}_bert_1.log python bench/bert_base_synth.py || exit 1
tail -1 gpurun_out/${tag}_pytest.log
for f in rn_off_1 rn_on_1 rn_off_2 rn_on_2 bert_1; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log | tail -1)"; done
echo SESSION_DONE
