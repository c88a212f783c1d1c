#!/usr/bin/env python3
"""List the kernels of a rocprofv3 results DB and flag library GEMM / convolution
kernels (hipBLASLt/Tensile ``Cijk_*``, rocBLAS, MIOpen) -- the check that a workload's
training step runs on cloud_amd's own kernels.

usage: lib_kernel_check.py <results.db> [--out summary.txt]   (exit 1 if any flagged)
"""
import argparse
import collections
import re
import sqlite3

LIB = re.compile(r"Cijk_|rocblas|miopen|MIOpen|naive_conv|igemm|gridwise|ck_tile|ck::|Tensile|batched_transpose",
                 re.I)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = sqlite3.connect(a.db).execute("select name, duration from kernels").fetchall()
    tot, cnt = collections.Counter(), collections.Counter()
    for name, dur in rows:
        k = re.sub(r"\(.*", "", name.replace("void ", "").replace("(anonymous namespace)::", ""))
        tot[k] += dur
        cnt[k] += 1
    flagged = [k for k in tot if LIB.search(k)]
    lines = [f"{len(rows)} dispatches, {len(tot)} distinct kernels, {len(flagged)} library GEMM/conv kernels"]
    for k, v in tot.most_common():
        lines.append(f"{'LIB ' if k in flagged else '    '}{v / 1e6:9.3f} ms {cnt[k]:6d}x  {k[:160]}")
    text = "\n".join(lines)
    print(text)
    if a.out:
        open(a.out, "w").write(text + "\n")
    raise SystemExit(1 if flagged else 0)


if __name__ == "__main__":
    main()
