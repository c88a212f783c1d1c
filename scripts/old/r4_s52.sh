#!/usr/bin/env bash
# Round-4 session 52: HBM bytes of the deep fused gradient kernel (FETCH_SIZE / WRITE_SIZE, one
# counter group per pass), stage-1 conv3 shape.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-r4s52}
rm -rf gpurun_out/${tag}_fetch gpurun_out/${tag}_write
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/${tag}_fetch -o run --output-format csv -- python bench/xa_dw_bench.py --batch 1024 --iters 3 > gpurun_out/${tag}_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/${tag}_write -o run --output-format csv -- python bench/xa_dw_bench.py --batch 1024 --iters 3 > gpurun_out/${tag}_write.log 2>&1 || exit 1
python3 - "$tag" <<'PY' > gpurun_out/${tag}_bytes.txt
import csv, glob, sys, collections
tag = sys.argv[1]
for kind in ("fetch", "write"):
    files = glob.glob(f"gpurun_out/{tag}_{kind}/**/*counter_collection.csv", recursive=True)
    agg = collections.defaultdict(list)
    for f in files:
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            if "xa_dw" not in name:
                continue
            agg[(name[:90], row.get("Counter_Name"))].append(float(row.get("Counter_Value", 0)))
    for (k, c), v in sorted(agg.items()):
        print(kind, c, f"calls={len(v)}", f"median_KB={sorted(v)[len(v)//2]:.0f}", k)
PY
rm -rf gpurun_out/${tag}_fetch gpurun_out/${tag}_write
cat gpurun_out/${tag}_bytes.txt
echo SESSION_DONE
