set -o pipefail
mkdir -p gpurun_out/s8
S=scripts/gpu_step.sh
for v in 0 1 2 3; do
  CLOUD_AMD_PRWN_VARIANT=$v CLOUD_AMD_SMALLK_SET=conv3 $S 200 s8/sk_v$v.log python -u bench/smallk_gemm.py || exit 1
done
CLOUD_AMD_PRWN_VARIANT=1 $S 300 s8/test_prw_v1.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_prw_gpu.py || exit 1
