#!/usr/bin/env python3
"""Kernel micro-benchmark for profiling: times one op of the hot path in isolation on the C2
workload (or a given size) with HIP events; used with rocprofv3 --pmc and ablation builds."""
import argparse, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd"))
import numpy as np
import torch
from insite_amd import ops, cohort

ap = argparse.ArgumentParser()
ap.add_argument("--op", default="gram", choices=["gram", "sindy_fit", "rollout", "stlsq"])
ap.add_argument("--patients", type=int, default=100_000)
ap.add_argument("--T", type=int, default=200)
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--method", default="rk4")
ap.add_argument("--layout", default="patient", choices=["patient", "time", "time_bits"])
a = ap.parse_args()
dev = torch.device("cuda:0")
xlay = "time" if a.layout == "time_bits" else a.layout
coh = cohort.synthetic_pkpd(a.patients, a.T, seed=1, device=dev, equation="EQ_4_C", layout=xlay)
lib = coh.lib
ws = ops.Workspace()
coef = torch.zeros((2, lib.n_terms), dtype=torch.float64, device=dev)
coef[0, 4] = -1.11; coef[1, 1] = -0.146; coef[1, 5] = -1.02
arm_cf = cohort.counterfactual_arms(coh.arm, a.T, seed=1, layout=a.layout)
y = torch.empty((a.patients, a.T) if a.layout == "patient" else (a.T, a.patients), dtype=torch.float64, device=dev)
G = torch.randn(a.patients, 7, 7, dtype=torch.float64, device=dev)
G = G @ G.transpose(1, 2) + torch.eye(7, dtype=torch.float64, device=dev) * 7
bb = torch.randn(a.patients, 7, dtype=torch.float64, device=dev)
def run():
    if a.op == "gram":
        ops.gram(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 2, "smoothed4", ws, layout=xlay)
    elif a.op == "sindy_fit":
        ops.sindy_fit(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, 100, True, 2, "smoothed4", ws,
                      layout=xlay)
    elif a.op == "rollout":
        ops.rollout(coh.y0, coh.u, arm_cf, coef, lib, coh.dt, method=a.method, T=a.T, out=y,
                    layout=a.layout)
    else:
        ops.stlsq(G, bb, 0.1, 0.5)
for _ in range(5): run()
torch.cuda.synchronize()
st = torch.cuda.current_stream()
e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
e0.record(st)
for _ in range(a.iters): run()
e1.record(st); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / a.iters
print(json.dumps({"op": a.op, "patients": a.patients, "T": a.T, "ms_per_call": ms,
                  "layout": a.layout, "lib": os.environ.get("INSITE_LIB_OVERRIDE", "default")}))
