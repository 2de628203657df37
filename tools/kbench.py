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
ap.add_argument("--op", default="gram", choices=["gram", "sindy_fit", "rollout", "stlsq", "step", "gram_seg", "fused",
                                                "deferred"])
ap.add_argument("--patients", type=int, default=100_000)
ap.add_argument("--T", type=int, default=200)
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--method", default="rk4")
ap.add_argument("--layout", default="patient", choices=["patient", "time", "time_bits"])
ap.add_argument("--cold", action="store_true",
                help="evict L2/Infinity Cache before every call and time each call alone")
ap.add_argument("--flush", default="read", choices=["read", "write"],
                help="cold eviction by reading 512 MB (clean cache) or writing it (dirty lines left behind)")
ap.add_argument("--timing", action="store_true", help="phase timestamps (needs an INSITE_TIMING build)")
ap.add_argument("--hwid", action="store_true", help="with --timing: wave end times by XCC / SE / CU")
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
step_out = (torch.empty((2, lib.n_terms), dtype=torch.float64, device=dev),
            torch.empty((2, lib.n_terms), dtype=torch.int8, device=dev), torch.empty(2, dtype=torch.int32, device=dev),
            torch.empty((2, lib.n_terms, lib.n_terms), dtype=torch.float64, device=dev),
            torch.empty((2, lib.n_terms), dtype=torch.float64, device=dev))
if a.op == "gram_seg":   # F4: 4-arm treatment-segment Gram, time-major (bench.py --config f4 cohort)
    seg = cohort.synthetic_segments(a.patients, a.T, seed=31, device=dev,
                                    coef=[[0, .2, 0, 0], [0, 0, 0, -.6], [0, -.3, 0, 0], [0, -.25, 0, -.9]])
if a.op == "fused":   # the fused step kernel (insite_fit_rollout_f64): discovery of coh | bit-arm rollout of coh
    fplan = ops.plan_fit_rollout(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, coh.y0, coh.u, arm_cf, coef,
                                 coh.dt, method=a.method, T=a.T, y_out=y, out=step_out, workspace=ws)
if a.op == "deferred":   # the deferred fused step (insite_fit_rollout_deferred_f64), slots alternating
    dws = ops.Workspace()
    dplans = [ops.plan_fit_rollout_deferred(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, coh.y0, coh.u,
                                            arm_cf, coef, coh.dt, j, True, dws, method=a.method, T=a.T, y_out=y,
                                            out=step_out) for j in range(2)]
    dpos = [0]
def run():
    if a.op == "fused":
        fplan()
        return
    if a.op == "deferred":
        dplans[dpos[0] % 2]()
        dpos[0] += 1
        return
    if a.op == "gram_seg":
        ops.gram_segments(seg.x, seg.arm, seg.seq_len, seg.u, seg.dt, seg.lib, 4, "order1", ws, layout="time")
    elif a.op == "gram":
        ops.gram(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 2, "smoothed4", ws, layout=xlay)
    elif a.op == "sindy_fit":
        ops.sindy_fit(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, 100, True, 2, "smoothed4", ws,
                      layout=xlay)
    elif a.op == "rollout":
        ops.rollout(coh.y0, coh.u, arm_cf, coef, lib, coh.dt, method=a.method, T=a.T, out=y,
                    layout=a.layout)
    elif a.op == "step":   # one bench step: discovery (gram + finalize/STLSQ) then the rollout
        ops.sindy_fit(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, 100, True, 2, "smoothed4", ws,
                      layout=xlay, out=step_out)
        ops.rollout(coh.y0, coh.u, arm_cf, step_out[0], lib, coh.dt, method=a.method, T=a.T, out=y, layout=a.layout)
    else:
        ops.stlsq(G, bb, 0.1, 0.5)
for _ in range(5): run()
torch.cuda.synchronize()
st = torch.cuda.current_stream()
if a.cold:
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    evs = []
    for i in range(a.iters):
        if a.flush == "write":
            flush.fill_(i & 0xff)
        else:
            fsum = flush.view(torch.float32).sum()
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st); run(); e1.record(st)
        evs.append((e0, e1))
    torch.cuda.synchronize()
    ms = float(np.mean([x.elapsed_time(y_) for x, y_ in evs]))
else:
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(a.iters): run()
    e1.record(st); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
if a.timing:
    import ctypes
    from insite_amd import _lib
    fn = _lib.load().insite_debug_tstamps
    buf = np.zeros((1 << 16) * 10, dtype=np.uint64)
    fn(ctypes.c_void_p(buf.ctypes.data), 1)
    torch.cuda.synchronize()
    for _ in range(3):
        if a.cold:   # the stamps of the last call, taken with L2 / Infinity Cache evicted before it
            fsum = flush.view(torch.float32).sum()
        run()
    torch.cuda.synchronize()
    fn(ctypes.c_void_p(buf.ctypes.data), 0)
    ts_all = buf.reshape(-1, 10).astype(np.int64)
    rbase = None
    for part, ts in (("gram", ts_all[:32768]), ("rollout", ts_all[32768:49152]), ("finalize", ts_all[49152:])):
        t = ts[ts[:, 0] > 0]
        if not len(t):
            continue
        out = {"kernel": part, "waves": len(t)}
        if a.hwid and part in ("gram", "rollout"):   # end time by where the wave ran (slot 7: HW_ID | XCC_ID << 32)
            hw = t[:, 7].astype(np.uint64)
            xcc = (hw >> np.uint64(32)).astype(np.int64) & 15
            cu = (hw >> np.uint64(8)).astype(np.int64) & 15
            se = (hw >> np.uint64(13)).astype(np.int64) & 7
            endt = (t[:, 9] - t[:, 8]) / 100.0
            out["end_by_xcc_us"] = {int(x): round(float(endt[xcc == x].mean()), 2) for x in np.unique(xcc)}
            out["end_by_se_us"] = {int(x): round(float(endt[se == x].mean()), 2) for x in np.unique(se)}
            cuid = xcc * 1000 + se * 100 + cu
            per_cu = np.array([endt[cuid == c].mean() for c in np.unique(cuid)])
            out["cu_mean_end_pcts"] = [round(float(np.percentile(per_cu, q)), 2) for q in (0, 10, 50, 90, 100)]
            out["within_cu_spread_us_mean"] = round(float(np.mean([endt[cuid == c].max() - endt[cuid == c].min()
                                                                   for c in np.unique(cuid)])), 2)
        for j in range(1, 7):
            ok = t[:, j] > 0
            if ok.any():
                out[f"slot{j}_cyc"] = round(float((t[ok, j] - t[ok, 0]).mean()))
        r0, r1 = t[:, 8], t[:, 9]
        okr = (r0 > 0) & (r1 > 0)
        r0, r1 = r0[okr], r1[okr]
        if rbase is None:
            rbase = r0.min()
        q = lambda v: [round(float(np.percentile(v, x)) / 100, 2) for x in (0, 10, 50, 90, 100)]
        out["start_us_pcts"] = q(r0 - rbase)
        out["end_us_pcts"] = q(r1 - rbase)
        out["dur_us_pcts"] = q(r1 - r0)
        print(json.dumps(out))
print(json.dumps({"op": a.op, "patients": a.patients, "T": a.T, "ms_per_call": ms,
                  "layout": a.layout, "cold": (a.flush if a.cold else False), "lib": os.environ.get("INSITE_LIB_OVERRIDE", "default")}))
