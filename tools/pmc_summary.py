"""Summarise a rocprofv3 --pmc CSV: mean counter value per dispatch, per kernel.

    python tools/pmc_summary.py OUT_DIR > summary.json
"""
import csv
import glob
import json
import sys
from collections import defaultdict

files = glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True)
acc = defaultdict(lambda: defaultdict(list))
for f in files:
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "?")
            acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
out = {}
for name, cs in acc.items():
    short = name if len(name) < 90 else name[:90]
    out[short] = {c: {"mean": sum(v) / len(v), "n": len(v)} for c, v in cs.items()}
print(json.dumps(out, indent=1))
