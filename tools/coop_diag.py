"""Diagnose the cooperative dense refinement against the single-lane kernel (prints where they differ)."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd"))
from insite_amd import cohort, ops
F4 = [[0.0, 0.20, 0.0, 0.0], [0.0, 0.0, 0.0, -0.60], [0.0, -0.30, 0.0, 0.0], [0.0, -0.25, 0.0, -0.90]]
dev = torch.device("cuda", 0)
N, T = int(os.environ.get("DIAG_N", 3000)), 60
coh = cohort.synthetic_segments(N, T, seed=N + 11, device=dev, coef=F4, dt=0.1)
V = coh.x[:T, :N].t().contiguous(); arm = coh.arm[:, :N].t().contiguous()
g = torch.Generator(device=dev); g.manual_seed(N)
sl = torch.randint(1, T + 1, (N,), generator=g, device=dev, dtype=torch.int32)
base = np.array(F4) * 1.1; c0 = np.where(base != 0, base, 0.01)
lib = coh.lib
if os.environ.get("DIAG_JOINT") == "1":
    from insite_amd.library import polynomial_library
    lib = polynomial_library(1, 2, True, n_inputs=2)
    c0 = np.array([[-0.36, 0.33, 0.49, 0.074, 0.80, -0.45, -0.45, -0.29, 0.19, -1.15, -0.34]])
outs = {}
for coop in ("1", "0"):
    os.environ["INSITE_REFINE_COOP"] = coop
    nf = torch.empty((N,), dtype=torch.int32, device=dev)
    r = ops.insite_refine(V, arm, coh.u, sl, c0, lib, coh.dt, 10.0, 5, nfev=nf)
    torch.cuda.synchronize()
    outs[coop] = [t.cpu().numpy() for t in r] + [nf.cpu().numpy()]
a, b = outs["1"], outs["0"]
names = ["preds", "coef", "status", "iters", "nfev"]
for n, x, y in zip(names, a, b):
    x = x.reshape(N, -1).astype(np.float64); y = y.reshape(N, -1).astype(np.float64)
    bad = np.where(~np.all((x == y) | (np.isnan(x) & np.isnan(y)), axis=1))[0]
    print(n, "rows differing", bad.size, "max abs", float(np.nanmax(np.abs(x - y))) if bad.size else 0.0, "first", bad[:8])
sl_h = sl.cpu().numpy()
bad = np.where(~np.all(a[0] == b[0], axis=1))[0]
print("sl of differing rows", sl_h[bad[:10]], "status", a[2][bad[:10]], b[2][bad[:10]], "nfev", a[4][bad[:10]], b[4][bad[:10]])
