#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV passes (run_counter_collection.csv) per kernel family.

usage: pmc_summary.py <pass_dir> [<pass_dir> ...]
Derived columns (gfx950 conventions, MI355X_MICROARCH.md):
  clk_MHz   = GRBM_GUI_ACTIVE / 8 / duration      (GRBM counts summed over 8 XCDs)
  mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
  HBM GB/s  = (FETCH_SIZE + WRITE_SIZE) KiB / duration  (FETCH_SIZE under-counts wide
              coalesced reads by up to 2x on gfx950 -- read it as a lower bound)
  lds_conf  = SQ_LDS_BANK_CONFLICT cycles per SQ_INSTS_LDS instruction
"""
import collections
import csv
import os
import re
import sys

csv.field_size_limit(1 << 30)


def family(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("ca::", "")
    m = re.match(r"([\w:]+?)<([^()]*?)>\(", n)
    if m:
        base = m.group(1).split("::")[-1]
        args = m.group(2)
        if "glds" in base or "wide" in base:
            parts = [a.strip() for a in args.split(",")]
            return f"{base}<{parts[0]}x{parts[1]},{parts[-1]}>"
        return base
    return re.sub(r"\(.*", "", n).split("::")[-1][:50]


def main(dirs):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(dict)
    seen = collections.defaultdict(set)  # counter -> passes that collected it
    for d in dirs:
        with open(os.path.join(d, "run_counter_collection.csv")) as f:
            for r in csv.DictReader(f):
                k = family(r["Kernel_Name"])
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                seen[r["Counter_Name"]].add(d)
                dur[k][(d, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    # a counter collected in several passes (GRBM_GUI_ACTIVE as the clock reference) is the
    # per-pass mean, so it stays comparable with counters collected once
    for k in acc:
        for cn, ds in seen.items():
            if len(ds) > 1 and cn in acc[k]:
                acc[k][cn] /= len(ds)
    rows = []
    for k, c in acc.items():
        t = sum(dur[k].values()) / max(1, len(dirs))  # each pass re-runs the same dispatches
        n = len(dur[k]) / max(1, len(dirs))
        g = c.get("GRBM_GUI_ACTIVE", 0.0)
        clk = g / 8 / t / 1e6 if t and g else float("nan")
        mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (g / 8 * 1024) if g else float("nan")
        hbm = (c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) * 1024 / t / 1e9 if t else float("nan")
        lds = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_INSTS_LDS"] if c.get("SQ_INSTS_LDS") else float("nan")
        rows.append((t, k, n, clk, mfma, hbm, lds))
    rows.sort(reverse=True)
    print(f"{'kernel family':58s} {'calls':>6s} {'ms':>8s} {'clk_MHz':>8s} {'mfma_util':>9s} {'HBM_GB/s':>9s} {'lds_conf':>8s}")
    for t, k, n, clk, mfma, hbm, lds in rows[:30]:
        print(f"{k[:58]:58s} {n:6.0f} {t * 1e3:8.2f} {clk:8.0f} {mfma:9.3f} {hbm:9.0f} {lds:8.2f}")


if __name__ == "__main__":
    main(sys.argv[1:])
