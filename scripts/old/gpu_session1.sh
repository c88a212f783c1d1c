#!/usr/bin/env bash
# GPU session 1: kernel numerics, smoke, first native + stock ResNet-50 numbers, rocprof.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 120 env.log python -c "import torch;print(torch.cuda.get_device_name(0), torch.version.hip)" || exit 1
$S 600 pytest_gpu.log python -m pytest tests -m gpu -x -q || exit 1
$S 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S 400 bench_native.log python bench.py --steps 10 --warmup 5 || exit 1
$S 400 stock_nhwc_amp.log python bench/stock_resnet50.py --steps 10 --warmup 5 --layout nhwc --precision amp || exit 1
$S 400 stock_nchw_amp.log python bench/stock_resnet50.py --steps 10 --warmup 5 --layout nchw --precision amp || exit 1
$S 400 stock_nhwc_bf16.log python bench/stock_resnet50.py --steps 10 --warmup 5 --layout nhwc --precision bf16 || exit 1
$S 500 prof_native.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_native -o run --output-format csv -- python bench.py --steps 5 --warmup 3 || exit 1
echo SESSION_DONE
