#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: mean counter value per dispatch for each kernel (KB units for
FETCH_SIZE / WRITE_SIZE)."""
import csv, glob, json, os, sys
from collections import defaultdict

root = sys.argv[1]
out = {}
for f in sorted(glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True)):
    run = os.path.relpath(f, root).split(os.sep)[0]
    acc = defaultdict(list)
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if "at::" in name or "rocclr" in name:
            continue
        key = (name.replace("void (anonymous namespace)::", "").split("(")[0], r["Counter_Name"])
        acc[key].append(float(r["Counter_Value"]))
    for (k, c), v in acc.items():
        out.setdefault(run, {})[f"{k} {c}"] = {"dispatches": len(v), "mean": sum(v) / len(v)}
print(json.dumps(out, indent=1))
