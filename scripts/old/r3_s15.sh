#!/usr/bin/env bash
# Round-3 session 15: two-rows-per-trip LayerNorm backward (BERT), ResNet-50 with the
# row-parallel loss kernel restored, native Keras pads / split-K bias+act, full GPU suite,
# MNIST fit profile, tuner.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s15}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 300 ${tag}_t1.log python -u -m pytest tests/test_transformer_gpu.py tests/test_bert_hf_parity.py tests/test_keras_native_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_t1.log
for i in 1 2; do
$S 240 ${tag}_bert_${i}.log python bench/bert_base_synth.py || exit 1
$S 240 ${tag}_bench_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
done
$S 900 ${tag}_pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_pytest.log
rm -rf gpurun_out/${tag}_prof_bert
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_prof_bert.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_bert -o run --output-format csv -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof_bert adam_kernel > gpurun_out/${tag}_bert_step_kernels.txt
rm -rf gpurun_out/${tag}_prof_bert
head -40 gpurun_out/${tag}_bert_step_kernels.txt
rm -rf gpurun_out/${tag}_prof_mnist
CLOUD_AMD_EXAMPLE_SMALL=1 $S 300 ${tag}_prof_mnist.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_mnist -o run --output-format csv -- python examples/workloads/mnist_example_using_fit.py || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof_mnist adam_kernel 8 > gpurun_out/${tag}_mnist_step_kernels.txt
rm -rf gpurun_out/${tag}_prof_mnist
head -3 gpurun_out/${tag}_mnist_step_kernels.txt
$S 400 ${tag}_tuner.log python bench/tuner_8trials.py || exit 1
for f in bert_1 bert_2 bench_1 bench_2 tuner; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log)"; done
echo SESSION_DONE
