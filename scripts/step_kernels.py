"""Per-step kernel summary from a rocprofv3 kernel trace: steps are delimited by the last
occurrence of a marker kernel (the optimizer); prints the mean per-step time per kernel
name, dispatch counts, and the kernel sequence of the last complete step.
usage: step_kernels.py <trace dir> <marker substring> [steps_to_skip]"""
import csv
import glob
import os
import sys
from collections import Counter, defaultdict


def main(d, marker, skip=3):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # step boundaries: after the last marker dispatch of a run of markers
    ends = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"] and
            (i + 1 == len(rows) or marker not in rows[i + 1]["Kernel_Name"])]
    steps = [(ends[k] + 1, ends[k + 1] + 1) for k in range(len(ends) - 1)][skip:]
    if not steps:
        print("no steps found")
        return
    tot = defaultdict(float)
    cnt = Counter()
    for a, b in steps:
        for r in rows[a:b]:
            n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:100]
            tot[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            cnt[n] += 1
    ns = len(steps)
    allms = sum(tot.values()) / ns
    print("steps %d, %.3f ms/step kernel time, %.1f dispatches/step" % (ns, allms, sum(cnt.values()) / ns))
    for n, t in sorted(tot.items(), key=lambda kv: -kv[1]):
        print("%9.3f ms/step %7.1f calls/step  %s" % (t / ns, cnt[n] / ns, n))
    a, b = steps[-1]
    print("\n--- sequence of the last step ---")
    for r in rows[a:b]:
        print("%8.1f us  %s" % ((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r["Kernel_Name"][:110]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 1)
