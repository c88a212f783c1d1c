#!/usr/bin/env bash
# Round-5 session 1: CTL gradient contract, optimizer-owned run-ahead bound, comm-init deadline;
# full GPU suite; ResNet-50 bench via run(); BERT bench + final-tree BERT step profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s1}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 600 ${tag}_new.log python -u -m pytest tests/test_ctl_gpu.py tests/test_comm_init_deadline.py tests/test_step_pacer_gpu.py tests/test_rccl_dataplane_gpu.py tests/test_workloads_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
chk ${tag}_new.log
$S 1200 ${tag}_all.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
chk ${tag}_all.log
$S 300 ${tag}_rn.log python bench.py --steps 20 --warmup 5 || exit 1
$S 300 ${tag}_bert.log python bench/bert_base_synth.py --steps 20 --warmup 5 || exit 1
rm -rf gpurun_out/${tag}_bprof
$S 300 ${tag}_bprof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_bprof -o run --output-format csv -- python bench/bert_base_synth.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_bprof adam_kernel > gpurun_out/${tag}_bert_step_kernels.txt || true
rm -rf gpurun_out/${tag}_bprof
tail -3 gpurun_out/${tag}_all.log
for f in gpurun_out/${tag}_rn.log gpurun_out/${tag}_bert.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
head -12 gpurun_out/${tag}_bert_step_kernels.txt
echo SESSION_DONE
