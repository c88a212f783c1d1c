#!/usr/bin/env bash
# Round-4 session 8: 256 cores in one process (ring v256, 8-phase p8 schedule 0 / 1, glds128) on
# random operands with fp32-reference numerics, twice; then one counter pass (clock, MFMA busy,
# wait split, LDS conflicts) of the 256 cores at 8192^3 next to hipBLASLt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-r4s8}
out=gpurun_out/$tag; mkdir -p $out
shapes="4096,4096,4096,0 8192,8192,8192,0 8192,2304,768,0 8192,768,3072,0 8192,3072,768,0 8192,8192,8192,1 8192,8192,8192,2"
for i in 1 2; do
timeout -k 10 240 bin/gemm_bench 20 $shapes > $out/gemm_bench_$i.txt 2>&1 || { echo "gemm_bench failed"; cat $out/gemm_bench_$i.txt; exit 1; }
done
cat $out/gemm_bench_1.txt $out/gemm_bench_2.txt
bash scripts/r3_pmc_gemm.sh ${tag}_pmc 8192,8192,8192,0 v256,p8s2,p8s4 || exit 1
echo SESSION_DONE
