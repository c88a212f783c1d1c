#!/usr/bin/env bash
# Round-3 session 9: deferred side-stream join + per-stream batched finalisation (BERT A/B),
# transformer tests, then a ResNet-50 b1024 serialized per-step kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r3s9}
$S 400 ${tag}_pytest.log python -u -m pytest tests/test_transformer_gpu.py tests/test_ddp_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/${tag}_pytest.log && ! grep -qE " failed| error" gpurun_out/${tag}_pytest.log || { echo "GPU tests failed"; tail -40 gpurun_out/${tag}_pytest.log; exit 1; }
$S 240 ${tag}_bert.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_GRAD_FIN_BATCH=0 $S 240 ${tag}_bert_f0.log python bench/bert_base_synth.py || exit 1
$S 240 ${tag}_bert2.log python bench/bert_base_synth.py || exit 1
CLOUD_AMD_GRAD_FIN_BATCH=0 $S 240 ${tag}_bert_f0b.log python bench/bert_base_synth.py || exit 1
rm -rf gpurun_out/${tag}_prof_rn
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_prof_rn.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof_rn -o run --output-format csv -- python bench.py --via-run 0 --steps 4 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof_rn sgd_kernel > gpurun_out/${tag}_rn_step_kernels.txt
head -50 gpurun_out/${tag}_rn_step_kernels.txt
for f in bert bert_f0 bert2 bert_f0b; do echo "$f $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_$f.log)"; done
echo SESSION_DONE
