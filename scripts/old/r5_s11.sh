#!/usr/bin/env bash
# Round-5 session 11: halo weight gradient (64 x 576 partial in registers per persistent
# workgroup), dgrad statistics loads issued mid-loop; numerics, shape timing, ResNet-50 A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
tag=${1:-r5s11}
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$S 300 ${tag}_t.log $PT tests/test_conv_halo_gpu.py tests/test_bn_fold_gpu.py || exit 1
grep -q "FAILED\|Error" gpurun_out/${tag}_t.log && { echo T_FAILED; tail -40 gpurun_out/${tag}_t.log; exit 1; }
grep -E "passed|failed" gpurun_out/${tag}_t.log
$S 120 ${tag}_cs.log python bench/conv_shapes.py l1_c2 1024 || exit 1
CLOUD_AMD_CONV_HALO_WGRAD=0 $S 120 ${tag}_cs_w0.log python bench/conv_shapes.py l1_c2 1024 || exit 1
grep -h tag gpurun_out/${tag}_cs.log gpurun_out/${tag}_cs_w0.log
for r in 1 2; do
$S 200 ${tag}_rn_h1_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_CONV_HALO_WGRAD=0 $S 200 ${tag}_rn_w0_$r.log python bench.py --steps 20 --warmup 5 || exit 1
CLOUD_AMD_CONV_HALO=0 $S 200 ${tag}_rn_h0_$r.log python bench.py --steps 20 --warmup 5 || exit 1
done
for f in gpurun_out/${tag}_rn_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | tail -1)"; done
CLOUD_AMD_WGRAD_STREAM=0 $S 300 ${tag}_rprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_rprof -o run --output-format csv -- python bench.py --via-run 0 --steps 5 --warmup 3 || exit 1
python3 scripts/step_kernels.py gpurun_out/${tag}_rprof sgd_kernel > gpurun_out/${tag}_rn_step_kernels.txt 2>&1 || true
head -3 gpurun_out/${tag}_rn_step_kernels.txt
grep -E "halo|splitk" gpurun_out/${tag}_rn_step_kernels.txt | head -12
echo SESSION_DONE
