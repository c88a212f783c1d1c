#!/usr/bin/env bash
# Round-4 session 34: the space-to-depth stem on tall 256 x 64 tiles (CLOUD_AMD_STEM_TALL).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r4s34}
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
CLOUD_AMD_STEM_TALL=1 $S 300 ${tag}_stem.log python -u -m pytest tests/test_stem_tail_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
chk ${tag}_stem.log
for r in 1 2; do
$S 240 ${tag}_rn_default_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_STEM_TALL=1 $S 240 ${tag}_rn_tall_${r}.log python bench.py --via-run 0 --steps 20 --warmup 5 || exit 1
done
rm -rf gpurun_out/${tag}_prof
CLOUD_AMD_STEM_TALL=1 CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_prof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_prof sgd_kernel > gpurun_out/${tag}_rn_step_kernels.txt
rm -rf gpurun_out/${tag}_prof
tail -1 gpurun_out/${tag}_stem.log
grep -n "GConvRowA" gpurun_out/${tag}_rn_step_kernels.txt | head -3
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
echo SESSION_DONE
