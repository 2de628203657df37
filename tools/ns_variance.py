#!/usr/bin/env python3
"""North-star step timing variance probe (diagnostic): in ONE process, the north_star_step workload timed on two
allocations of its cohorts (regenerated between), each timed twice; run several processes to separate within-process
from between-process variance.  Prints one JSON line per process."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd"))
import torch  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prealloc", action="store_true", help="reserve 24 GB in the caching allocator first")
    ap.add_argument("--soak", type=int, default=0,
                    help="after the first allocation's two timings, this many more launches on it, then time it again "
                         "(a clock / power-state ramp shows up as a faster third timing on the SAME allocation)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if a.prealloc:
        blk = torch.empty((24 << 30) // 8, dtype=torch.float64, device=dev)
        del blk
    from insite_amd import cohort
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    ns = argparse.Namespace(**vars(args))
    ns.patients, ns.T, ns.steps, ns.warmup, ns.dstreams, ns.gram_blocks = 1_000_000, 500, 20, 3, 1, 0
    out = []
    for alloc in range(2):
        sd = [1900 + 10 * alloc, 1901 + 10 * alloc]
        cohs = [cohort.synthetic_pkpd(1_000_000, 500, seed=s_, device=dev, equation="EQ_4_C", layout="time") for s_ in sd]
        arms = [cohort.counterfactual_arms(c.arm, 500, seed=s_, layout="time_bits") for c, s_ in zip(cohs, sd)]
        torch.cuda.synchronize(dev)
        for rep in range(2 if not (a.soak and alloc == 0) else 3):
            if rep == 2:   # soak: a.soak launches on the same allocation (untimed), then the third timing
                ns2 = argparse.Namespace(**vars(ns))
                ns2.warmup, ns2.steps = a.soak, 2
                t0 = time.perf_counter()
                bench.deferred_run(ns2, dev, cohs[0], arms[0], cohs[1], arms[1])
                out.append({"soak_launches": a.soak, "soak_s": round(time.perf_counter() - t0, 3)})
            fr = bench.deferred_run(ns, dev, cohs[0], arms[0], cohs[1], arms[1])
            out.append({"alloc": alloc, "rep": rep, "ms_step": round(fr["ms_step"], 5), "launch_ms": round(fr["step_ms"], 5)})
            del fr
        del cohs, arms
        torch.cuda.empty_cache()
    print(json.dumps({"prealloc": a.prealloc, "soak": a.soak, "runs": out}), flush=True)


if __name__ == "__main__":
    main()
