#!/bin/bash
# GEMM core A/B on one MI355X: bin/gemm_bench (all in-tree cores, numerics vs fp32 reference)
# then the hipBLASLt comparator on the same shapes.  Usage: scripts/r3_gemm.sh <tag> [shapes...]
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
shapes="$@"
[ -z "$shapes" ] && shapes="4096,4096,4096,0 8192,8192,8192,0 4096,4096,4096,1 4096,4096,4096,2 8192,2304,768,0 8192,3072,768,0 8192,768,3072,0 8192,768,768,0 8192,768,3072,1 768,3072,8192,2"
timeout -k 10 240 bin/gemm_bench 20 $shapes > $out/gemm_bench.txt 2>&1 || { echo "gemm_bench failed rc=$?"; cat $out/gemm_bench.txt; exit 1; }
cat $out/gemm_bench.txt
timeout -k 10 400 python bench/blas_ref.py $shapes > $out/blas.txt 2>&1 || { echo "blas_ref failed"; cat $out/blas.txt; exit 1; }
cat $out/blas.txt
