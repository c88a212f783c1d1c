#!/usr/bin/env bash
# Round-4 session 44: stem-tail pooling kernels with their window loads ahead of any branch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s44}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 300 ${tag}_stem.log python -u -m pytest tests/test_stem_tail_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_stem.log
CLOUD_AMD_STEM_BWD_RECOMPUTE=1 $S 300 ${tag}_stem_rc.log python -u -m pytest tests/test_stem_tail_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_stem_rc.log
rm -rf gpurun_out/${tag}_prof
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_prof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof sgd_kernel > gpurun_out/${tag}_rn_step_kernels.txt
rm -rf gpurun_out/${tag}_prof
rm -rf gpurun_out/${tag}_prof2
CLOUD_AMD_STEM_BWD_RECOMPUTE=1 CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_prof2.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof2 -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof2 sgd_kernel > gpurun_out/${tag}_rn_step_kernels_recompute.txt
rm -rf gpurun_out/${tag}_prof2
for r in 1 2; do
$S 240 ${tag}_rn_default_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_STEM_BWD_RECOMPUTE=1 $S 240 ${tag}_rn_rc_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
done
tail -1 gpurun_out/${tag}_stem.log
grep -n "maxpool\|bn_bwd_apply_kernel<false" gpurun_out/${tag}_rn_step_kernels.txt | head -4
grep -n "maxpool" gpurun_out/${tag}_rn_step_kernels_recompute.txt | head -4
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
