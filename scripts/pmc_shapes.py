"""Per-(kernel, grid) summary of one rocprofv3 --pmc pass (run_counter_collection.csv).

usage: python scripts/pmc_shapes.py <counter_collection.csv> [top]
Columns: fraction of wave cycles parked on s_waitcnt/barrier (SQ_WAIT_ANY), issue-stalled
(SQ_WAIT_INST_ANY) and issuing (SQ_ACTIVE_INST_ANY); MFMA pipe busy share (SQ_VALU_MFMA_BUSY_CYCLES
over GRBM_GUI_ACTIVE/8 x 1024 SIMDs); VALU and SALU instructions per wave.
"""
import collections
import csv
import re
import sys

csv.field_size_limit(1 << 30)
path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows, meta = collections.defaultdict(dict), {}
for r in csv.DictReader(open(path)):
    d = int(r["Dispatch_Id"])
    rows[d][r["Counter_Name"]] = float(r["Counter_Value"])
    meta[d] = (r["Kernel_Name"], int(r["Grid_Size"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "").replace("ca::", "")
    return re.sub(r"\(.*", "", n)[:75]


agg = collections.defaultdict(collections.Counter)
for d, c in rows.items():
    name, grid, dur = meta[d]
    a = agg[(short(name), grid)]
    a["n"] += 1
    a["dur"] += dur
    for k, v in c.items():
        a[k] += v
print("%-75s %8s %5s %7s %6s %6s %6s %6s %7s %6s" % ("kernel", "grid", "n", "us", "wait", "winst", "actv", "mfma%",
                                                    "valu/w", "salu/w"))
for (name, grid), a in sorted(agg.items(), key=lambda kv: -kv[1]["dur"])[:top]:
    wc = a["SQ_WAVE_CYCLES"] or 1
    clk = a["GRBM_GUI_ACTIVE"] / 8
    nw = grid / 64
    print("%-75s %8d %5d %7.1f %6.2f %6.2f %6.2f %6.1f %7.0f %6.0f" % (
        name, grid, a["n"], a["dur"] / a["n"] / 1e3, a["SQ_WAIT_ANY"] / wc, a["SQ_WAIT_INST_ANY"] / wc,
        a["SQ_ACTIVE_INST_ANY"] / wc, 100 * a["SQ_VALU_MFMA_BUSY_CYCLES"] / (clk * 1024) if clk else 0,
        a["SQ_INSTS_VALU"] / a["n"] / nw, a["SQ_INSTS_SALU"] / a["n"] / nw))
