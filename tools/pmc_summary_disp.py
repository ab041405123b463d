"""Summarise a rocprofv3 --pmc CSV per dispatch GROUP: kernels of the same name are split
into consecutive groups of 20 dispatches (one group per case of the driver), mean per group.

    python tools/pmc_summary_disp.py OUT_DIR > summary.json
"""
import csv
import glob
import json
import sys
from collections import defaultdict

files = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)
rows = []
for f in files:
    with open(f) as fh:
        rows.extend(csv.DictReader(fh))
by = defaultdict(lambda: defaultdict(float))
order = []
for r in rows:
    key = (r.get("Kernel_Name", "?")[:60], int(r.get("Dispatch_Id", 0)))
    if key not in by:
        order.append(key)
    by[key][r["Counter_Name"]] += float(r["Counter_Value"])
order.sort(key=lambda k: k[1])
out = []
GROUP = int(sys.argv[2]) if len(sys.argv) > 2 else 20
for i in range(0, len(order), GROUP):
    keys = order[i:i + GROUP]
    agg = defaultdict(float)
    for k in keys:
        for c, v in by[k].items():
            agg[c] += v / len(keys)
    out.append({"kernel": keys[0][0], "first_dispatch": keys[0][1], "n": len(keys), **{c: round(v) for c, v in agg.items()}})
print(json.dumps(out, indent=1))
