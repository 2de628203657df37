"""Probe (tooling, not product): where the C5 line's ms_per_step exceeds its per-launch event time.  Same cohort
as bench.py c5_main; times (a) the bench's loop (wall clock around K plan() calls), (b) one event pair around that
loop, (c) per-call event pairs, (d) the rollout alone with the order precomputed, (e) the plan captured in a
hipGraph (one graph launch per step).  Run: python tools/probe/c5_gap.py"""
import os
import ctypes
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd"))
import bench  # noqa: E402
from insite_amd import ops, cohort  # noqa: E402
from insite_amd.library import polynomial_library  # noqa: E402

dev = torch.device("cuda:0")
N, K = 1_000_000, 20
g = torch.Generator(device=dev)
g.manual_seed(5)
t_obs, n_obs = cohort.irregular_grid(N, seed=4, device=dev)
Tm = t_obs.size(0)
t_dev = torch.nan_to_num(t_obs, nan=0.0).t().contiguous()
u = torch.randn((N, 2), generator=g, device=dev, dtype=torch.float64) * 0.05 + 0.5
y0 = torch.rand((N,), generator=g, device=dev, dtype=torch.float64) * 49 + 1
arm = (torch.rand((N, Tm), generator=g, device=dev) < 0.5).to(torch.int8)
bits = ops.pack_arm_bits(arm, Tm)
lib = polynomial_library(2, 2, True)
coef = torch.zeros((2, lib.n_terms), dtype=torch.float64, device=dev)
coef[0, 4], coef[1, 1], coef[1, 5] = bench.C5_COEF
y = torch.empty((N, (Tm + 7) // 8 * 8), dtype=torch.float64, device=dev)[:, :Tm]
steps = torch.empty((N,), dtype=torch.int32, device=dev)
plan = ops.plan_rollout_rk45(y0, u, bits, t_dev, n_obs, coef, lib, out=y, steps=steps, layout="patient", order=True)
order = ops.rk45_order(n_obs, Tm)
plan_r = ops.plan_rollout_rk45(y0, u, bits, t_dev, n_obs, coef, lib, out=y, steps=steps, layout="patient",
                               order=order)
st = torch.cuda.current_stream(dev)


def wall(fn):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K * 1e3


def ev_loop(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(st)
    for _ in range(K):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / K


def ev_each(fn):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    for a, b in evs:
        a.record(st)
        fn()
        b.record(st)
    torch.cuda.synchronize()
    return float(np.mean([a.elapsed_time(b) for a, b in evs]))


def host_submit(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / K * 1e3


order_b = torch.empty_like(order)
ws_b = torch.zeros((1 << 17,), dtype=torch.float64, device=dev)
L = ops._lib.load()
oargs = (ops._p(n_obs), N, int(Tm), ops._p(order_b), ops._p(ws_b), ws_b.numel() * 8)


def order_into_b():
    st_ = L.insite_rk45_order_i32(*oargs, ctypes.c_void_p(st.cuda_stream))
    assert st_ == 0


plan_b = ops.plan_rollout_rk45(y0, u, bits, t_dev, n_obs, coef, lib, out=y, steps=steps, layout="patient",
                               order=order_b)
order_c = order.clone()
plan_c = ops.plan_rollout_rk45(y0, u, bits, t_dev, n_obs, coef, lib, out=y, steps=steps, layout="patient",
                               order=order_c)


def dummy_then_fixed():      # the order kernels into a buffer the rollout does not read, then the fixed order
    order_into_b()
    plan_r()


def fresh_then_rollout():    # the order kernels into order_b, the rollout on order_b (= plan)
    order_into_b()
    plan_b()


def copy_then_rollout():     # the fixed order re-written (a 4 MB copy) just before the rollout reads it
    order_c.copy_(order)
    plan_c()


for name, fn in (("plan", plan), ("rollout_only", plan_r), ("order_only", lambda: ops.rk45_order(n_obs, Tm)),
                 ("dummy+fixed", dummy_then_fixed), ("fresh+rollout", fresh_then_rollout),
                 ("copy+rollout", copy_then_rollout), ("order_b_only", order_into_b)):
    print(f"{name:13s} wall {wall(fn):.4f}  ev_loop {ev_loop(fn):.4f}  ev_each {ev_each(fn):.4f}  "
          f"host_submit {host_submit(fn):.4f} ms", flush=True)
print(f"plan again    wall {wall(plan):.4f}  ev_each {ev_each(plan):.4f}", flush=True)
