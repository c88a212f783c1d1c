#!/usr/bin/env bash
# Round-6 session 35: final-tree evidence -- full GPU suite + smoke, ResNet-50 x3, BERT x3,
# serialized step profiles of both, world-2 shared-GPU rehearsals (gloo) with the DP A/B cells.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s35
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 1000 ${tag}_all.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs || exit 1
chk ${tag}_all.log
tail -2 gpurun_out/${tag}_all.log
$S 300 ${tag}_smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" || exit 1
tail -1 gpurun_out/${tag}_smoke.log
for r in 1 2 3; do
$S 200 ${tag}_rn_$r.log python bench.py --steps 20 --warmup 5 || exit 1
$S 200 ${tag}_bert_$r.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_rn_*.log gpurun_out/${tag}_bert_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
rm -rf gpurun_out/${tag}_rprof
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_rprof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_rprof -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_rprof sgd_kernel > gpurun_out/${tag}_rn_step_kernels.txt || true
rm -rf gpurun_out/${tag}_rprof
head -3 gpurun_out/${tag}_rn_step_kernels.txt
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_bprof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_bprof -o run --output-format csv -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_bprof adam_kernel > gpurun_out/${tag}_bert_step_kernels.txt || true
rm -rf gpurun_out/${tag}_bprof
head -3 gpurun_out/${tag}_bert_step_kernels.txt
export CLOUD_AMD_JOBS_DIR=$PWD/gpurun_out/${tag}_jobs
export CLOUD_AMD_SHARED_GPU=1 CLOUD_AMD_DIST_BACKEND=gloo CLOUD_AMD_NUM_GPUS=2
$S 400 ${tag}_rn_dp2.log python bench.py --gpus 2 --steps 5 --warmup 3 --batch 128 || exit 1
$S 400 ${tag}_bert_dp2.log python bench/bert_base_synth.py --gpus 2 --steps 5 --warmup 3 || exit 1
rm -rf gpurun_out/${tag}_jobs
for f in gpurun_out/${tag}_*dp2.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1) $(grep -o '"replicas_consistent": [a-z]*' $f | tail -1) cells=$(grep -o '"exposed_comm_ms"' $f | wc -l)"; done
echo SESSION_DONE
