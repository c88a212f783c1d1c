"""Summarise a rocprofv3 --kernel-trace --pmc run per kernel name: mean duration, effective
clock (GRBM_GUI_ACTIVE / 8 XCDs / duration), MFMA-busy fraction (SQ_VALU_MFMA_BUSY_CYCLES
over the CU-cycles of the dispatch) and the SQ wave-state split.  usage: pmc_clock.py <dir>"""
import csv
import glob
import os
import sys
from collections import defaultdict


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main(d):
    for sub in sorted(glob.glob(os.path.join(d, "*"))):
        if not os.path.isdir(sub):
            continue
        ctr = rows(os.path.join(sub, "**", "*counter_collection.csv"))
        if not ctr:
            continue
        agg = defaultdict(lambda: defaultdict(float))
        durs = defaultdict(list)
        kt = {}
        for r in rows(os.path.join(sub, "**", "*kernel_trace.csv")):
            cid = r.get("Correlation_Id") or r.get("Dispatch_Id")
            try:
                kt[cid] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            except (KeyError, ValueError):
                pass
        for r in ctr:
            name = r.get("Kernel_Name", "?")[:90]
            cid = r.get("Correlation_Id") or r.get("Dispatch_Id")
            agg[(name, cid)][r["Counter_Name"]] += float(r["Counter_Value"])
            if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                durs[(name, cid)] = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])]
            elif cid in kt:
                durs[(name, cid)] = [kt[cid]]
        per = defaultdict(list)
        for (name, cid), c in agg.items():
            dur = durs.get((name, cid), [0])[0]
            per[name].append((c, dur))
        print("==", os.path.basename(sub))
        for name, lst in sorted(per.items(), key=lambda kv: -sum(x[1] for x in kv[1])):
            n = len(lst)
            dur = sum(x[1] for x in lst) / n
            c = defaultdict(float)
            for cc, _ in lst:
                for k, v in cc.items():
                    c[k] += v / n
            clk = c["GRBM_GUI_ACTIVE"] / 8 / dur if dur else 0  # cycles per ns = GHz
            cu_cycles = c["GRBM_GUI_ACTIVE"] / 8 * 256
            mfma = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (cu_cycles * 4) if cu_cycles else 0
            wc = c["SQ_WAVE_CYCLES"] or 1
            nm = c["SQ_VALU_MFMA_BUSY_CYCLES"]
            print("   mfma_busy_cycles=%.3g gui_active/8=%.3g" % (nm, c["GRBM_GUI_ACTIVE"] / 8))
            print("%-90s n=%3d dur=%8.1fus clk=%.2fGHz mfma_busy=%.3f wait_any=%.2f wait_inst=%.2f active=%.2f "
                  "lds_conf/inst=%.2f lds_conf/idx_active=%.3f" % (name, n, dur / 1e3, clk, mfma, c["SQ_WAIT_ANY"] / wc,
                                          c["SQ_WAIT_INST_ANY"] / wc, c["SQ_ACTIVE_INST_ANY"] / wc,
                                          c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_INSTS_LDS"], 1),
                                          c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_LDS_IDX_ACTIVE"], 1)))


if __name__ == "__main__":
    main(sys.argv[1])
