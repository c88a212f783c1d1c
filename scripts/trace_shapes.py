"""Per-(kernel, grid) time breakdown from a rocprofv3 kernel_trace.csv.

usage: python scripts/trace_shapes.py <run_kernel_trace.csv> <steps> [name-filter] [top]
"""
import csv
import re
import sys
from collections import defaultdict

path, steps = sys.argv[1], float(sys.argv[2])
filt = sys.argv[3] if len(sys.argv) > 3 else ""
top = int(sys.argv[4]) if len(sys.argv) > 4 else 40
agg = defaultdict(lambda: [0.0, 0])
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"]
    if filt and filt not in name:
        continue
    short = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))
    short = short.replace("void ", "")[:110]
    key = (short, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["VGPR_Count"], r["LDS_Block_Size"])
    agg[key][0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    agg[key][1] += 1
rows = sorted(agg.items(), key=lambda kv: -kv[1][0])
tot = sum(v[0] for v in agg.values())
print("total %.3f ms/step" % (tot / steps))
for (k, gx, gy, gz, vg, lds), (ms, n) in rows[:top]:
    print("%8.3f ms/step %5.1f calls  avg %7.1f us  grid=%s,%s,%s vgpr=%s lds=%s  %s" % (
        ms / steps, n / steps, 1000 * ms / n, gx, gy, gz, vg, lds, k))
