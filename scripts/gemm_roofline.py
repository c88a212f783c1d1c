"""Per-call roofline of the GEMM / convolution launches of a serialized run.

usage: python scripts/gemm_roofline.py <kernel_trace.csv | results.db> <shape_log.jsonl> [PF/s] [TB/s]

The shape log (CLOUD_AMD_SHAPE_LOG, written by cloud_amd.ops.raw) lists every GEMM-class
launch in order; the trace's GEMM-class kernels (dense_gemm*/conv_glds*/mfma*, plus the
split-K reduce that follows a weight gradient) are matched to it from the END of both
sequences (the log also holds the untraced warm-up / first-step launches).  Floor of a call =
max(2*M*N*K / peak_flops, min_bytes / hbm_bw); the table shows where the time above the
floor sits, by launch kind and per call.
"""
import csv
import json
import sys
from collections import defaultdict

trace, logp = sys.argv[1], sys.argv[2]
PF = float(sys.argv[3]) if len(sys.argv) > 3 else 1.3e15
BW = float(sys.argv[4]) if len(sys.argv) > 4 else 5.5e12

if trace.endswith(".db"):
    import sqlite3

    rows = [dict(Kernel_Name=n, Start_Timestamp=a, End_Timestamp=b) for n, a, b in
            sqlite3.connect(trace).execute("select name, start, end from kernels")]
else:
    rows = list(csv.DictReader(open(trace)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def is_body(n):
    return ("dense_gemm" in n or "conv_glds" in n or "gemm_pp" in n) and "reduce" not in n


calls = []  # [name, us, extra_us]
for r in rows:
    n = r["Kernel_Name"]
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if is_body(n):
        calls.append([n.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:90], us, 0.0])
    elif "splitk_reduce" in n and calls:
        calls[-1][2] += us
log = [json.loads(l) for l in open(logp)]


def role(name):
    fam = "dense" if "dense_gemm" in name else "conv"
    if "WgradB" in name or name.count("GDenseNC") == 2:
        return "wgrad", fam
    if "Dgrad" in name or "GDenseKC, ca::GDenseNC" in name:
        return "dgrad", fam
    return "fwd", fam


def lrole(kind):
    fam = "dense" if (kind.startswith("dense") or kind.endswith("1x1") or "1x1s1" in kind or "1x1_" in kind) else "conv"
    if kind == "dense_nn":
        return "dgrad", fam
    return ("wgrad" if "wgrad" in kind else ("dgrad" if "dgrad" in kind else "fwd")), fam


# Walk both sequences from the end.  A log entry may own several kernels (strided dgrad:
# one per output-parity class); a kernel whose role (fwd / dgrad / wgrad, from its loader
# types) disagrees with the entry is an unlogged launch (e.g. a Keras Dense layer) and skipped.
merged, ci, skipped = [], len(calls) - 1, 0.0
for e in reversed(log):
    k = e.get("launches", 4 if (e["kind"].startswith("dgrad") and "s2" in e["kind"]) else 1)
    while ci >= 0 and role(calls[ci][0]) != lrole(e["kind"]):
        skipped += calls[ci][1] + calls[ci][2]
        ci -= 1
    if ci - k + 1 < 0:
        break
    grp = calls[ci - k + 1:ci + 1]
    ci -= k
    merged.append([grp[0][0], sum(g[1] for g in grp), sum(g[2] for g in grp)])
n = len(merged)
calls, log = merged[::-1], log[-n:]
print("unmatched kernels skipped: %.2f ms" % (skipped / 1e3))
agg = defaultdict(lambda: [0, 0.0, 0.0, 0.0])
per = []
for (name, us, red), e in zip(calls, log):
    fl = 2.0 * e["M"] * e["N"] * e["K"]
    floor = max(fl / PF, e["bytes"] / BW) * 1e6
    t = us + red
    a = agg[e["kind"]]
    a[0] += 1
    a[1] += t
    a[2] += floor
    a[3] += fl
    per.append((t - floor, t, floor, e, name, red))
tot_t = sum(a[1] for a in agg.values())
tot_f = sum(a[2] for a in agg.values())
print("matched %d calls; measured %.2f ms, floor %.2f ms (PF %.2f, BW %.1f TB/s)" % (
    n, tot_t / 1e3, tot_f / 1e3, PF / 1e15, BW / 1e12))
print("%-18s %6s %10s %10s %8s %8s" % ("kind", "calls", "ms", "floor_ms", "x_floor", "TF/s"))
for k, (c, t, f, fl) in sorted(agg.items(), key=lambda kv: -(kv[1][1] - kv[1][2])):
    print("%-18s %6d %10.2f %10.2f %8.2f %8.0f" % (k, c, t / 1e3, f / 1e3, t / max(f, 1e-9), fl / t / 1e6))
print("\nby shape (mean per call, all calls):")
shp = defaultdict(lambda: [0, 0.0, 0.0, 0.0])
for ex, t, f, e, name, red in per:
    a = shp[(e["kind"], e["M"], e["N"], e["K"], e.get("splits", 0))]
    a[0] += 1
    a[1] += t
    a[2] += f
    a[3] += red
print("%-14s %8s %6s %9s %6s %6s %9s %9s %7s %8s" % ("kind", "M", "N", "K", "splits", "calls", "us", "floor_us", "x_flr",
                                                     "over_ms"))
for (kind, m, nn, kk, sp), (c, t, f, red) in sorted(shp.items(), key=lambda kv: -(kv[1][1] - kv[1][2])):
    print("%-14s %8d %6d %9d %6d %6d %9.1f %9.1f %7.2f %8.2f" % (kind, m, nn, kk, sp, c, t / c, f / c, t / f,
                                                                (t - f) / 1e3))
print("\ntop calls by time above floor:")
for ex, t, f, e, name, red in sorted(per, key=lambda p: -p[0])[:40]:
    print("%7.1f us over (%7.1f vs floor %7.1f, reduce %5.1f) %-14s M=%d N=%d K=%d %s %s" % (
        ex, t, f, red, e["kind"], e["M"], e["N"], e["K"], ("splits=%d" % e["splits"]) if "splits" in e else "", name))
