#!/usr/bin/env bash
# Round-3 session 17: strided-row one-block loss kernel, which torch ops remain in a Keras
# step (profiler attribution), MNIST fit kernel profile, tuner throughput, and counter passes
# on the final ResNet-50 tree (b256, serialized, kernel trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s17}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 300 ${tag}_t1.log python -u -m pytest tests/test_keras_native_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_t1.log
$S 200 ${tag}_keras_ops.log python scripts/debug/keras_step_ops.py || exit 1
head -40 gpurun_out/${tag}_keras_ops.log
rm -rf gpurun_out/${tag}_prof_mnist
CLOUD_AMD_EXAMPLE_SMALL=1 $S 300 ${tag}_prof_mnist.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_mnist -o run --output-format csv -- python examples/workloads/mnist_example_using_fit.py || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof_mnist adam_kernel 8 > gpurun_out/${tag}_mnist_step_kernels.txt
rm -rf gpurun_out/${tag}_prof_mnist
head -3 gpurun_out/${tag}_mnist_step_kernels.txt
$S 400 ${tag}_tuner_1.log python bench/tuner_8trials.py || exit 1
$S 400 ${tag}_tuner_2.log python bench/tuner_8trials.py || exit 1
B="python bench.py --via-run 0 --steps 2 --warmup 1 --batch 256"
CLOUD_AMD_WGRAD_STREAM=0 $S 200 ${tag}_pmc1.log timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv \
  -d gpurun_out/${tag}_pmc1 -o run --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- $B || exit 1
CLOUD_AMD_WGRAD_STREAM=0 $S 200 ${tag}_pmc2.log timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv \
  -d gpurun_out/${tag}_pmc2 -o run --pmc FETCH_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -- $B || exit 1
CLOUD_AMD_WGRAD_STREAM=0 $S 200 ${tag}_pmc3.log timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv \
  -d gpurun_out/${tag}_pmc3 -o run --pmc WRITE_SIZE GRBM_GUI_ACTIVE -- $B || exit 1
python3 scripts/pmc_summary.py gpurun_out/${tag}_pmc1 gpurun_out/${tag}_pmc2 gpurun_out/${tag}_pmc3 > gpurun_out/${tag}_pmc_summary.txt 2>&1
head -30 gpurun_out/${tag}_pmc_summary.txt
rm -rf gpurun_out/${tag}_pmc1 gpurun_out/${tag}_pmc2 gpurun_out/${tag}_pmc3
for f in tuner_1 tuner_2; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log)"; done
echo SESSION_DONE
