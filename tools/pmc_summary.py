"""Summarise a rocprofv3 --pmc counter_collection CSV per kernel: dispatches and mean counter value
per dispatch.   python tools/pmc_summary.py <dir> <out.json>"""
import csv
import glob
import json
import os
import re
import sys

rows = {}
for path in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    with open(path) as f:
        for r in csv.DictReader(f):
            name = re.sub(r"\(anonymous namespace\)::", "", r.get("Kernel_Name", ""))
            name = name.split("(")[0].replace("void ", "").strip()
            ctr = r.get("Counter_Name", "")
            val = float(r.get("Counter_Value", 0.0))
            e = rows.setdefault(name, {}).setdefault(ctr, [0, 0.0])
            e[0] += 1
            e[1] += val
out = {k: {c: {"dispatches": n, "mean": s / max(n, 1), "total": s} for c, (n, s) in v.items()} for k, v in rows.items()}
json.dump(out, open(sys.argv[2], "w"), indent=1)
top = sorted(out.items(), key=lambda kv: -max(x["total"] for x in kv[1].values()))[:12]
for k, v in top:
    print(k, {c: (x["dispatches"], round(x["mean"], 1)) for c, x in v.items()})
