#!/usr/bin/env bash
# Round-3 session 13: deeper LDS-DMA rings for the N = 64 persistent GEMMs (A/B vs the tiled
# core), ResNet-50 A/B, serialized ResNet-50 b1024 per-step kernel profile with the core;
# plain-GEMM engine policy (auto vs in-tree only) on BERT-base.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s13}
$S 300 ${tag}_prw_test.log python -u -m pytest tests/test_gemm_prw_gpu.py tests/test_plain_gemm_policy_gpu.py tests/test_keras_native_gpu.py -x -v --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/${tag}_prw_test.log && ! grep -qE " failed| error" gpurun_out/${tag}_prw_test.log || { echo "PRW test failed"; tail -60 gpurun_out/${tag}_prw_test.log; exit 1; }
CLOUD_AMD_GEMM_PRW=1 $S 300 ${tag}_smallk_prw1.log python bench/smallk_gemm.py || exit 1
CLOUD_AMD_GEMM_PRW=0 $S 300 ${tag}_smallk_prw0.log python bench/smallk_gemm.py || exit 1
grep -h '"M"' gpurun_out/${tag}_smallk_prw1.log gpurun_out/${tag}_smallk_prw0.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['prw'], r['M'], r['K'], r['N'], 'stats', r['ours_stats_us'], 'plain', r['ours_us'])"
for i in 1 2; do
$S 240 ${tag}_bench_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_GEMM_PRW=0 $S 240 ${tag}_bench_prw0_${i}.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
done
rm -rf gpurun_out/${tag}_prof_rn
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_prof_rn.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_rn -o run --output-format csv -- python bench.py --via-run 0 --steps 4 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof_rn sgd_kernel > gpurun_out/${tag}_rn_step_kernels.txt
rm -rf gpurun_out/${tag}_prof_rn
head -50 gpurun_out/${tag}_rn_step_kernels.txt
for i in 1 2; do
$S 240 ${tag}_bert_${i}.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_GEMM_LIB=never $S 240 ${tag}_bert_never_${i}.log python bench/bert_base_synth.py || exit 1
done
grep -h -o '"plain_gemm_engine".*' gpurun_out/${tag}_bert_1.log
rm -rf gpurun_out/${tag}_prof_mnist
CLOUD_AMD_EXAMPLE_SMALL=1 $S 300 ${tag}_prof_mnist.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_mnist -o run --output-format csv -- python examples/workloads/mnist_example_using_fit.py || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof_mnist adam_kernel 8 > gpurun_out/${tag}_mnist_step_kernels.txt
rm -rf gpurun_out/${tag}_prof_mnist
head -40 gpurun_out/${tag}_mnist_step_kernels.txt
$S 400 ${tag}_tuner.log python bench/tuner_8trials.py || exit 1
CLOUD_AMD_TUNER_STANDBY=0 $S 400 ${tag}_tuner_nostandby.log python bench/tuner_8trials.py || exit 1
for f in bench_1 bench_prw0_1 bench_2 bench_prw0_2 bert_1 bert_never_1 bert_2 bert_never_2 tuner tuner_nostandby; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log)"; done
echo SESSION_DONE
