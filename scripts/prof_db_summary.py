#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd SQLite database (``*_results.db``) by kernel.

usage: prof_db_summary.py <results.db> <steps> [--top N] [--detail NAME_SUBSTR]
Prints ms/step per kernel (short name) and, with --detail, the per-dispatch
grid/duration table of the matching kernels (to map launches to shapes).
"""
import argparse
import collections
import re
import sqlite3


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    n = n.replace("void ", "")
    n = re.sub(r"<.*", "", n)
    return n.split("::")[-1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("steps", type=float)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--detail", default=None)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x, lds_size, vgpr_count, accum_vgpr_count from kernels").fetchall()
    tot = collections.Counter()
    calls = collections.Counter()
    for r in rows:
        k = short(r[0])
        tot[k] += r[1]
        calls[k] += 1
    allns = sum(tot.values())
    print(f"total {allns / a.steps / 1e6:.3f} ms/step ({a.steps:g} steps, {len(rows)} dispatches)")
    for k, v in tot.most_common(a.top):
        print(f"{v / a.steps / 1e6:9.3f} ms/step {calls[k] / a.steps:8.1f} calls/step  {k}")
    if a.detail:
        agg = collections.defaultdict(list)
        for r in rows:
            if a.detail in short(r[0]):
                agg[(short(r[0]),) + tuple(r[2:])].append(r[1])
        print("\nkernel grid(x,y,z) wg lds vgpr agpr : calls mean_us total_ms/step")
        for key, d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            print(f"{key} : {len(d)} {sum(d) / len(d) / 1e3:.1f} {sum(d) / a.steps / 1e6:.3f}")


if __name__ == "__main__":
    main()
