#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats kernel_stats.csv by kernel category (ms per step)."""
import collections
import csv
import sys


def cat(n):
    if n.startswith("Cijk") or n.startswith("Custom_Cijk"):
        return "hipblaslt"
    if n.startswith("igemm") or "miopen" in n.lower() or n.startswith("naive_conv") or "Op2dTensor" in n or n.startswith("MIOpen") or "batchnorm" in n.lower() or n.startswith("Sub"):
        return "miopen:" + n.split("(")[0][:40]
    if "anonymous namespace" in n:
        return "cloud_amd:" + n.split("::")[1].split("(")[0].split("<")[0]
    if n.startswith("void at::") or n.startswith("at::"):
        return "torch:" + n.split("<")[0].replace("void at::native::", "")[:40]
    return "other:" + n[:50]


def main(path, steps):
    rows = list(csv.DictReader(open(path)))
    c = collections.Counter()
    calls = collections.Counter()
    for r in rows:
        k = cat(r["Name"])
        c[k] += float(r["TotalDurationNs"]) / steps / 1e6
        calls[k] += int(r["Calls"]) / steps
    tot = sum(c.values())
    print(f"total {tot:.2f} ms/step over {steps} steps")
    for k, v in c.most_common():
        print(f"{v:8.3f} ms/step {calls[k]:7.1f} calls/step  {k}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0)
