#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r3_blasnames; mkdir -p $out
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $out -o blas --output-format csv -- python3 bench/blas_ref.py "$@" > $out/blas.log 2>&1 || { tail -20 $out/blas.log; exit 1; }
cat $out/blas.log
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r3_blasnames/**/*kernel_trace.csv", recursive=True):
    seen = {}
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "Cijk" in n or "gemm" in n.lower():
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            seen.setdefault(n, []).append((d, r["Grid_Size_X"], r["Workgroup_Size_X"], r["LDS_Block_Size"], r["VGPR_Count"]))
    for n, v in seen.items():
        print(len(v), n[:150], v[0])
PY
