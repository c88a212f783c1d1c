#!/usr/bin/env bash
# Round-4 session 3: BN-fold kernels (numerics + bitwise vs unfused), the 8-phase 256 core
# (numerics), RCCL data-plane tests; ResNet-50 fold A/B; GEMM core A/B (ring vs 8-phase);
# serialized ResNet step profile; BERT.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s3}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 400 ${tag}_new.log python -u -m pytest tests/test_rccl_dataplane_gpu.py tests/test_transformer_gpu.py -k "dataplane or rccl or raising" -x -v -s --timeout 120 --timeout-method thread || exit 1
chk ${tag}_new.log
for i in 1 2; do
CLOUD_AMD_BN_FOLD=0 CLOUD_AMD_BN_FOLD_FWD=0 $S 240 ${tag}_rn_off_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 240 ${tag}_rn_on_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
done
CLOUD_AMD_BN_FOLD_FWD=0 $S 240 ${tag}_rn_bwdonly.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 300 ${tag}_gemm_ring.log python bench/gemm_core_ab.py || exit 1
CLOUD_AMD_GEMM_CORE=p8 $S 300 ${tag}_gemm_p8.log python bench/gemm_core_ab.py || exit 1
$S 240 ${tag}_bert_1.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_GEMM_CORE=p8 $S 240 ${tag}_bert_p8.log python bench/bert_base_synth.py || exit 1
rm -rf gpurun_out/${tag}_prof_rn
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_prof_rn.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_rn -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof_rn sgd_kernel > gpurun_out/${tag}_rn_step_kernels.txt
rm -rf gpurun_out/${tag}_prof_rn
head -30 gpurun_out/${tag}_rn_step_kernels.txt
for f in rn_off_1 rn_on_1 rn_off_2 rn_on_2 rn_bwdonly bert_1 bert_p8; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log | tail -1)"; done
grep summary gpurun_out/${tag}_gemm_ring.log gpurun_out/${tag}_gemm_p8.log
echo SESSION_DONE
