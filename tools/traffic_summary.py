#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 --pmc passes (tools/g_traffic.sh): for every config directory
<root>/<config>/{fetch,write}/**/counter_collection.csv, the MEDIAN per-dispatch FETCH_SIZE / WRITE_SIZE of
each product kernel (KiB in rocprofv3's derived counters), converted to bytes -- reads x the 8-B-per-lane
calibration of profiles/traffic_r02.json (FETCH_SIZE tallies 128-B streaming requests at 64 B,
MI355X_MICROARCH.md HBM section), writes exact.  Writes JSON {config: {kernel: {...}}} to stdout."""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

READ_FACTOR = 2.0   # profiles/traffic_r02.json calibration (tools/probe/layout_probe): 1.9996


def per_kernel(path_glob, counter):
    acc = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(path_glob, recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if "at::" in name or "rocclr" in name or r["Counter_Name"] != counter:
                continue
            k = name.replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "").split("(")[0]
            acc[(k, r.get("Grid_Size", ""))][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {key: list(d.values()) for key, d in acc.items()}


def main(root):
    out = {}
    for cdir in sorted(glob.glob(os.path.join(root, "*"))):
        if not os.path.isdir(cdir):
            continue
        cfg = os.path.basename(cdir)
        fe = per_kernel(os.path.join(cdir, "fetch", "**", "*counter_collection.csv"), "FETCH_SIZE")
        wr = per_kernel(os.path.join(cdir, "write", "**", "*counter_collection.csv"), "WRITE_SIZE")
        res = {}
        for key in sorted(set(fe) | set(wr)):
            k, grid = key
            f = statistics.median(fe[key]) if key in fe else None
            w = statistics.median(wr[key]) if key in wr else None
            rd = f * 1024 * READ_FACTOR if f is not None else None
            wb = w * 1024 if w is not None else None
            res[f"{k} grid={grid}"] = {
                "kernel": k, "grid_size": grid, "dispatches": max(len(fe.get(key, [])), len(wr.get(key, []))),
                "FETCH_SIZE_KiB_median": f, "WRITE_SIZE_KiB_median": w, "hbm_read_bytes": rd, "hbm_write_bytes": wb,
                "hbm_bytes": (rd or 0.0) + (wb or 0.0) if (rd is not None or wb is not None) else None}
        out[cfg] = res
    out["_method"] = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over the config's bench.py "
                      "line (tools/g_traffic.sh); median per dispatch; reads x 2.0 (8-B-per-lane calibration, "
                      "profiles/traffic_r02.json), writes exact")
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
