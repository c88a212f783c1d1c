"""GPU idle time per training step from a rocprofv3 kernel trace: steps delimited as in
step_kernels.py (after the last dispatch of the marker kernel); per step, wall = from the
step's first kernel start to its last kernel end, busy = the union of all kernel intervals
(every stream), idle = wall - busy -- the launch gaps and host stalls a graph capture or a
deeper queue could hide.  usage: step_idle.py <trace dir> <marker substring> [steps_to_skip]"""
import csv
import glob
import os
import sys


def main(d, marker, skip=3):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"] and
            (i + 1 == len(rows) or marker not in rows[i + 1]["Kernel_Name"])]
    steps = [(ends[k] + 1, ends[k + 1] + 1) for k in range(len(ends) - 1)][skip:]
    if not steps:
        print("no steps found")
        return
    out = []
    for a, b in steps:
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows[a:b])
        wall = max(e for _, e in iv) - iv[0][0]
        busy, cs, ce = 0, iv[0][0], iv[0][1]
        for s, e in iv[1:]:
            if s > ce:
                busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        out.append((wall / 1e6, busy / 1e6, (wall - busy) / 1e6, b - a))
    for w, bu, idle, n in out:
        print("wall %.3f ms  busy %.3f ms  idle %.3f ms  dispatches %d" % (w, bu, idle, n))
    k = len(out)
    print("mean: wall %.3f  busy %.3f  idle %.3f ms/step" % (sum(o[0] for o in out) / k, sum(o[1] for o in out) / k,
                                                        sum(o[2] for o in out) / k))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 1)
