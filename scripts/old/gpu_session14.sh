#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 600 pytest_gpu8.log env CLOUD_AMD_GEMM_CORE=glds8 python -m pytest tests/test_kernels_gpu.py tests/test_transformer_gpu.py -q -x || exit 1
$S 300 ab_glds8.log env CLOUD_AMD_GEMM_CORE=glds8 python bench/gemm_core_ab.py || exit 1
$S 300 ab_glds.log python bench/gemm_core_ab.py || exit 1
$S 300 conv8.log env CLOUD_AMD_GEMM_CORE=glds8 python bench/conv_shapes.py || exit 1
$S 400 bench8.log env CLOUD_AMD_GEMM_CORE=glds8 python bench.py --steps 20 --warmup 5 || exit 1
$S 400 bench_bert8.log env CLOUD_AMD_GEMM_CORE=glds8 python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
$S 400 bench.log python bench.py --steps 20 --warmup 5 || exit 1
$S 400 bench_bert.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
$S 300 pytest_ddp_gpu.log python -m pytest tests/test_ddp_gpu.py -q -x || exit 1
$S 500 prof_bert.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o run --output-format csv -- python bench/bert_base_synth.py --steps 5 --warmup 3 || exit 1
$S 300 graph.log python bench.py --graph 1 --steps 10 --warmup 3 || exit 1
echo SESSION_DONE
