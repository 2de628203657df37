#!/usr/bin/env python3
"""Per-dispatch view of a rocprofv3 kernel trace: durations and gaps of the INSITE kernels."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
sel = [r for r in rows if any(k in r["Kernel_Name"] for k in ("gram_kernel", "discovery_finalize", "rollout", "stlsq", "patient_fit", "sse"))]
first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
cnt = int(sys.argv[3]) if len(sys.argv) > 3 else 30
prev_end = None
for r in sel[first:first + cnt]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("void (anonymous namespace)::", "").split("(")[0]
    gap = (s - prev_end) / 1e3 if prev_end else 0
    print(f"{name[:60]:60s} grid={r.get('Grid_Size_X', r.get('Grid_Size',''))} dur={(e - s) / 1e3:8.2f}us gap={gap:7.2f}us")
    prev_end = e
