#!/usr/bin/env bash
# Round-3 session 19: Keras step without the zero-regularizer add and with one-launch padded
# gradient delivery (op attribution + MNIST fit kernel profile), and a counter pass over the
# BERT-base step (where LayerNorm backward / attention spend their cycles).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s19}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 300 ${tag}_t1.log python -u -m pytest tests/test_keras_native_gpu.py tests/test_dp_lockstep.py -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_t1.log
$S 200 ${tag}_keras_ops.log python scripts/debug/keras_step_ops.py || exit 1
grep -v amdgpu.ids gpurun_out/${tag}_keras_ops.log | head -30
rm -rf gpurun_out/${tag}_prof_mnist
CLOUD_AMD_EXAMPLE_SMALL=1 $S 300 ${tag}_prof_mnist.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_mnist -o run --output-format csv -- python examples/workloads/mnist_example_using_fit.py || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof_mnist adam_kernel 8 > gpurun_out/${tag}_mnist_step_kernels.txt
rm -rf gpurun_out/${tag}_prof_mnist
head -3 gpurun_out/${tag}_mnist_step_kernels.txt
$S 400 ${tag}_tuner.log python bench/tuner_8trials.py || exit 1
B="python bench/bert_base_synth.py --via-run 0 --steps 3 --warmup 2"
CLOUD_AMD_WGRAD_STREAM=0 $S 200 ${tag}_pmc1.log timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv \
  -d gpurun_out/${tag}_pmc1 -o run --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- $B || exit 1
CLOUD_AMD_WGRAD_STREAM=0 $S 200 ${tag}_pmc2.log timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv \
  -d gpurun_out/${tag}_pmc2 -o run --pmc FETCH_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -- $B || exit 1
CLOUD_AMD_WGRAD_STREAM=0 $S 200 ${tag}_pmc3.log timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv \
  -d gpurun_out/${tag}_pmc3 -o run --pmc WRITE_SIZE GRBM_GUI_ACTIVE -- $B || exit 1
python3 scripts/pmc_summary.py gpurun_out/${tag}_pmc1 gpurun_out/${tag}_pmc2 gpurun_out/${tag}_pmc3 > gpurun_out/${tag}_bert_pmc_summary.txt 2>&1
python3 scripts/pmc_dump.py gpurun_out/${tag}_pmc1 > gpurun_out/${tag}_bert_pmc1_dump.txt 2>&1 || true
head -30 gpurun_out/${tag}_bert_pmc_summary.txt
rm -rf gpurun_out/${tag}_pmc1 gpurun_out/${tag}_pmc2 gpurun_out/${tag}_pmc3
echo "tuner $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_tuner.log)"
echo SESSION_DONE
