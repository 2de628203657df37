#!/usr/bin/env python3
"""A/B helper (profiling only): the bench's north-star rollout (1M x 500 RK4, bench.py north_star_rollout) with
time-major and tile-major bit arms, events around each launch; one JSON line per layout.  Run once per library
(INSITE_LIB_OVERRIDE) and interleave."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd"))
import numpy as np
import torch
from insite_amd import ops, cohort

dev = torch.device("cuda:0")
N, T = int(os.environ.get("NSR_N", 1_000_000)), int(os.environ.get("NSR_T", 500))
lib = cohort.synthetic_pkpd(64, 8, seed=1, device=dev, equation="EQ_4_C", layout="time").lib
coef = torch.zeros((2, lib.n_terms), dtype=torch.float64, device=dev)
coef[0, 4] = -1.11; coef[1, 1] = -0.146; coef[1, 5] = -1.02
g = torch.Generator(device=dev); g.manual_seed(7)
y0 = torch.rand(N, generator=g, device=dev, dtype=torch.float64) * 49 + 1
u = torch.rand((N, 2), generator=g, device=dev, dtype=torch.float64) * 0.1 + 0.45
flip = torch.randint(0, T, (N, 1), generator=g, device=dev)
arm = (torch.arange(T, device=dev)[:, None] >= flip[:, 0][None, :]).to(torch.int8)
bits = ops.pack_arm_bits(arm, N)
tiles = ops.tile_major_bits(bits, N)
y = torch.empty((T, N), dtype=torch.float64, device=dev)
ref = None
for name, a in (("bits", bits), ("tiles", tiles)):
    for _ in range(5):
        ops.rollout(y0, u, a, coef, lib, 10.0 / T, method="rk4", out=y, layout="time_bits")
    evs = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); ops.rollout(y0, u, a, coef, lib, 10.0 / T, method="rk4", out=y, layout="time_bits"); e1.record()
        evs.append((e0, e1))
    torch.cuda.synchronize()
    ms = float(np.mean([p.elapsed_time(q) for p, q in evs]))
    cs = float(y[:, ::997].sum().item())
    if ref is None:
        ref = cs
    print(json.dumps({"lib": os.path.basename(os.environ.get("INSITE_LIB_OVERRIDE", "") or "default"), "arms": name,
                      "N": N, "T": T, "ms": ms, "frac": N * T * 8.125 / (ms * 1e-3) / 8e12, "checksum_equal": cs == ref}),
          flush=True)
