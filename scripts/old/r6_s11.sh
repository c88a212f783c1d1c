#!/usr/bin/env bash
# Round-6 session 11: 8-wave stem tile -- numerics, ResNet A/B, step profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s11
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 300 ${tag}_t.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stem_lds_gpu.py tests/test_kernels_gpu.py || exit 1
chk ${tag}_t.log
tail -2 gpurun_out/${tag}_t.log
for r in 1 2; do
$S 200 ${tag}_rn_on_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_STEM_LDS=0 $S 200 ${tag}_rn_off_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
rm -rf gpurun_out/${tag}_rprof
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_rprof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_rprof -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_rprof sgd_kernel > gpurun_out/${tag}_rn_step_kernels.txt || true
rm -rf gpurun_out/${tag}_rprof
head -12 gpurun_out/${tag}_rn_step_kernels.txt
echo SESSION_DONE
