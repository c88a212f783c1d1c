#!/usr/bin/env bash
# Round-3 session 21: full GPU suite on the pruned tree, attention forward at 3 blocks/CU
# (BERT bench + per-step profile), Keras step attribution + MNIST profile + tuner, BERT
# counter pass, ResNet-50 bench and serialized profile (stem max-pool loads issued up front).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s21}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 300 ${tag}_t1.log python -u -m pytest tests/test_kernels_gpu.py tests/test_transformer_gpu.py tests/test_bert_hf_parity.py tests/test_keras_native_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_t1.log
for i in 1 2; do
$S 240 ${tag}_bert_${i}.log python bench/bert_base_synth.py || exit 1
$S 240 ${tag}_bench_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
done
$S 900 ${tag}_pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_pytest.log
$S 200 ${tag}_keras_ops.log python scripts/debug/keras_step_ops.py || exit 1
grep -v amdgpu.ids gpurun_out/${tag}_keras_ops.log | head -30
rm -rf gpurun_out/${tag}_prof_mnist
CLOUD_AMD_EXAMPLE_SMALL=1 $S 300 ${tag}_prof_mnist.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_mnist -o run --output-format csv -- python examples/workloads/mnist_example_using_fit.py || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof_mnist adam_kernel 8 > gpurun_out/${tag}_mnist_step_kernels.txt
rm -rf gpurun_out/${tag}_prof_mnist
head -3 gpurun_out/${tag}_mnist_step_kernels.txt
$S 400 ${tag}_tuner.log python bench/tuner_8trials.py || exit 1
rm -rf gpurun_out/${tag}_prof_bert
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_prof_bert.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_bert -o run --output-format csv -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof_bert adam_kernel > gpurun_out/${tag}_bert_step_kernels.txt
rm -rf gpurun_out/${tag}_prof_bert
head -24 gpurun_out/${tag}_bert_step_kernels.txt
B="python bench/bert_base_synth.py --via-run 0 --steps 3 --warmup 2"
CLOUD_AMD_WGRAD_STREAM=0 $S 200 ${tag}_pmc1.log timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv \
  -d gpurun_out/${tag}_pmc1 -o run --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- $B || exit 1
CLOUD_AMD_WGRAD_STREAM=0 $S 200 ${tag}_pmc2.log timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv \
  -d gpurun_out/${tag}_pmc2 -o run --pmc FETCH_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -- $B || exit 1
CLOUD_AMD_WGRAD_STREAM=0 $S 200 ${tag}_pmc3.log timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv \
  -d gpurun_out/${tag}_pmc3 -o run --pmc WRITE_SIZE GRBM_GUI_ACTIVE -- $B || exit 1
python3 scripts/pmc_summary.py gpurun_out/${tag}_pmc1 gpurun_out/${tag}_pmc2 gpurun_out/${tag}_pmc3 > gpurun_out/${tag}_bert_pmc_summary.txt 2>&1
head -30 gpurun_out/${tag}_bert_pmc_summary.txt
rm -rf gpurun_out/${tag}_pmc1 gpurun_out/${tag}_pmc2 gpurun_out/${tag}_pmc3
rm -rf gpurun_out/${tag}_prof_rn
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_prof_rn.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_rn -o run --output-format csv -- python bench.py --via-run 0 --steps 4 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof_rn sgd_kernel > gpurun_out/${tag}_rn_step_kernels.txt
rm -rf gpurun_out/${tag}_prof_rn
grep -E "ms/step kernel|maxpool|stem" gpurun_out/${tag}_rn_step_kernels.txt | head -8
for f in bert_1 bert_2 bench_1 bench_2 tuner; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log)"; done
echo SESSION_DONE
