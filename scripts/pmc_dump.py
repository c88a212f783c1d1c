"""Mean of every counter per kernel name in a rocprofv3 counter_collection CSV tree."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
agg = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        per = defaultdict(lambda: defaultdict(float))
        for r in csv.DictReader(fh):
            per[(r["Kernel_Name"][:60], r.get("Correlation_Id") or r.get("Dispatch_Id"))][r["Counter_Name"]] += float(
                r["Counter_Value"])
        for (name, _), c in per.items():
            for k, v in c.items():
                agg[name][k].append(v)
for name, c in agg.items():
    print(name, {k: "%.4g" % (sum(v) / len(v)) for k, v in sorted(c.items())})
