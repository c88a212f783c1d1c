#!/usr/bin/env bash
# Round-3 session 11: Keras step glue removal (device-resident batches, fused metrics and
# zero_grad, by-value optimizer hyper-parameters, native Dropout / GlobalMaxPooling2D):
# GPU tests, MNIST fit per-step kernel profile, tuner bench, BERT + ResNet benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s11}
$S 700 ${tag}_pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/${tag}_pytest.log && ! grep -qE " failed| error" gpurun_out/${tag}_pytest.log || { echo "GPU tests failed"; tail -40 gpurun_out/${tag}_pytest.log; exit 1; }
rm -rf gpurun_out/${tag}_prof_mnist
CLOUD_AMD_EXAMPLE_SMALL=1 $S 300 ${tag}_prof_mnist.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_mnist -o run --output-format csv -- python examples/workloads/mnist_example_using_fit.py || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof_mnist adam_kernel 8 > gpurun_out/${tag}_mnist_step_kernels.txt
head -40 gpurun_out/${tag}_mnist_step_kernels.txt
$S 400 ${tag}_tuner.log python bench/tuner_8trials.py || exit 1
$S 240 ${tag}_bert.log python bench/bert_base_synth.py || exit 1
$S 240 ${tag}_bench.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
for f in bert bench tuner; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log)"; done
echo SESSION_DONE
