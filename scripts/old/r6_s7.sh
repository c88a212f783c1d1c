set -o pipefail
mkdir -p gpurun_out/s7
S=scripts/gpu_step.sh
$S 300 s7/test_prw.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_prw_gpu.py || exit 1
grep -q "passed" gpurun_out/s7/test_prw.log && ! grep -q "failed" gpurun_out/s7/test_prw.log || exit 1
CLOUD_AMD_SMALLK_SET=conv3 $S 200 s7/sk_on.log python -u bench/smallk_gemm.py || exit 1
CLOUD_AMD_SMALLK_SET=conv3 CLOUD_AMD_GEMM_PRWN=0 $S 200 s7/sk_off.log python -u bench/smallk_gemm.py || exit 1
$S 300 s7/rn_on_1.log python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_GEMM_PRWN=0 $S 300 s7/rn_off_1.log python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 300 s7/rn_on_2.log python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
CLOUD_AMD_GEMM_PRWN=0 $S 300 s7/rn_off_2.log python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
