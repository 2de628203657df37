"""Per-(kernel, grid) summary of a rocprofv3 --kernel-trace CSV.

rocprofv3 --stats averages every dispatch of a kernel symbol together; the C2 bench launches the same
rollout_tm_kernel instance for the 100k x 200 step (grid 391 x 256) and for the 1M x 500 north-star probe
(grid 3907 x 256), so the per-symbol average mixes two workloads.  This splits the same trace by grid size.

usage: python tools/rocprof_by_grid.py <kernel_trace.csv> [out.csv]
"""
import csv
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    m = re.match(r"(?:void\s+)?([\w:]+(?:<[^()]*>)?)", name)
    return m.group(1) if m else name[:120]


def main(path, out=None):
    rows = list(csv.DictReader(open(path)))
    if not rows:
        raise SystemExit("empty trace")
    keys = rows[0].keys()
    gx = next(k for k in keys if k.lower() in ("grid_size_x", "grid_size", "grid_sizex"))
    acc = defaultdict(list)
    for r in rows:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        acc[(short(r["Kernel_Name"]), int(r[gx]))].append(d)
    lines = [("kernel", "grid_threads_x", "calls", "avg_ns", "min_ns", "max_ns", "total_ns")]
    for (k, g), ds in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        lines.append((k, g, len(ds), round(sum(ds) / len(ds), 1), min(ds), max(ds), sum(ds)))
    w = csv.writer(open(out, "w", newline="") if out else sys.stdout)
    w.writerows(lines)


if __name__ == "__main__":
    main(*sys.argv[1:])
