#!/usr/bin/env bash
# Keras workloads on the native kernels: new GPU tests, then rocprof kernel traces of the
# reference MNIST fit workload and of the CIFAR tuner trial, checked for library kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 r2s5_pytest_keras.log python -u -m pytest tests/test_keras_native_gpu.py -v --timeout 120 --timeout-method thread || exit 1
CLOUD_AMD_EXAMPLE_SMALL=1 $S 300 r2s5_mnist_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/r2s5_mnist -o run -- python examples/workloads/mnist_example_using_fit.py || exit 1
python scripts/lib_kernel_check.py gpurun_out/r2s5_mnist/run_results.db --out gpurun_out/r2s5_mnist_kernels.txt > /dev/null; echo "mnist lib-check rc=$?" >> gpurun_out/session.log
echo SESSION_DONE
