#!/usr/bin/env bash
# BN-backward statistics in the dgrad epilogues: numerics + A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 pytest_new.log python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "bn_backward_stats or hands_off or fused_bottleneck or conv_fwd" || exit 1
grep -q " passed" gpurun_out/pytest_new.log && ! grep -q "FAILED\|ERROR" gpurun_out/pytest_new.log || { echo "new tests failed"; exit 1; }
$S 300 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
$S 300 bench_epi1.log python bench.py --steps 20 --warmup 5 || exit 1
$S 300 bench_epi0.log env CLOUD_AMD_BN_BWD_EPILOGUE=0 python bench.py --steps 20 --warmup 5 || exit 1
$S 300 bench_epi1_b256.log python bench.py --steps 20 --warmup 5 --batch 256 || exit 1
$S 300 bench_epi0_b256.log env CLOUD_AMD_BN_BWD_EPILOGUE=0 python bench.py --steps 20 --warmup 5 --batch 256 || exit 1
echo SESSION_DONE
