#!/usr/bin/env python3
"""Times insite_refine_arms_f64 (4 arms, EQ_5-like 4 x 7 model) at 6 / 12 / 28 active coefficients
(the M = 8, 16 and 36 kernels) on a synthetic cohort; profiling / tuning only (oracle cohort generator
as the data source, not a checker)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd"))
import numpy as np
import torch
from insite_amd import ops
from insite_amd.library import polynomial_library
from oracle import segments_ref as S

n = int(os.environ.get("N_ROWS", "200000"))
dev = torch.device("cuda:0")
rng = np.random.default_rng(5)
coef = np.zeros((4, 7))
coef[:, 1] = [0.2, -0.3, -0.25, 0.1]
coef[:, 4] = [-0.4, 0.0, -0.6, -0.2]
coef[1:, 5] = [0.3, -0.2, 0.25]
coef[::2, 0] = [0.05, -0.05]
x, u, arm, _ = S.synthetic_cohort(n, 60, rng, switch_p=0.1, noise=0.01, dt=1 / 6, coef=coef, n_statics=2)
V = torch.tensor(x[:, :60].copy(), device=dev)
A = torch.tensor(arm.astype(np.int8), device=dev)
U = torch.tensor(u, device=dev)
sl = torch.full((n,), 60, dtype=torch.int32, device=dev)
lib = polynomial_library(2, 2, True)
out = {}
for m in (6, 12, 28):
    c0 = coef * (1.0 + rng.normal(0.0, 0.1, size=coef.shape))
    flat = c0.reshape(-1)
    order = np.argsort(-np.abs(coef.reshape(-1)))
    keep = np.zeros(28, bool)
    keep[order[:m]] = True
    flat[~keep] = 0.0
    flat[keep & (np.abs(flat) <= 1e-3)] = 0.02
    c0 = flat.reshape(4, 7)
    for _ in range(2):
        r = ops.insite_refine(V, A, U, sl, c0, lib, 1 / 6, 10.0, 5)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        r = ops.insite_refine(V, A, U, sl, c0, lib, 1 / 6, 10.0, 5)
    e1.record()
    torch.cuda.synchronize()
    st = r[2].cpu().numpy()
    out[m] = {"ms": e0.elapsed_time(e1) / 3, "converged": float((st == 0).mean()),
              "iters": float(r[3].float().mean().item())}
print(json.dumps({"rows": n, "by_active": out}))
