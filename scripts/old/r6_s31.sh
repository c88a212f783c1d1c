#!/usr/bin/env bash
# Round-6 session 31: two-deep 16-wave transform-A tiles (CLOUD_AMD_XA_N256=3) -- bitwise tests,
# ResNet-50 A/B over the fold sites (default 128 vs 256 / 512 with the two-deep tiles), and a
# serialized profile of the 512 variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=r6s31
chk() { grep -q " passed" gpurun_out/$1 && ! grep -qE " failed| error" gpurun_out/$1 || { echo "tests failed: $1"; tail -60 gpurun_out/$1; exit 1; }; }
$S 400 ${tag}_kt.log python -u -m pytest tests/test_bn_fold_gpu.py -x -q --timeout 200 --timeout-method thread -k "wide_tiles or bnbwd_vs or bnapply_vs" || exit 1
chk ${tag}_kt.log
tail -1 gpurun_out/${tag}_kt.log
for r in 1 2; do
$S 200 ${tag}_rn_def_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD_MAX_N=512 CLOUD_AMD_XA_N256=3 $S 200 ${tag}_rn_n512d_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_BN_FOLD_MAX_N=256 CLOUD_AMD_XA_N256=3 $S 200 ${tag}_rn_n256d_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
rm -rf gpurun_out/${tag}_rprof
CLOUD_AMD_BN_FOLD_MAX_N=512 CLOUD_AMD_XA_N256=3 CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_rprof.log \
  rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_rprof -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_rprof sgd_kernel > gpurun_out/${tag}_rn_step_kernels_512d.txt || true
rm -rf gpurun_out/${tag}_rprof
head -3 gpurun_out/${tag}_rn_step_kernels_512d.txt
echo SESSION_DONE
