"""Profile target: the dense 4-arm INSITE refinement (the cooperative kernel) on PROF_N rows, PROF_REPS calls.

Prints the per-call time (HIP events) and the mean evaluation count; run under rocprofv3 --pmc for counters."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd"))
from insite_amd import cohort, ops
F4 = [[0.0, 0.20, 0.0, 0.0], [0.0, 0.0, 0.0, -0.60], [0.0, -0.30, 0.0, 0.0], [0.0, -0.25, 0.0, -0.90]]
dev = torch.device("cuda", 0)
N, T = int(os.environ.get("PROF_N", 200000)), 60
coh = cohort.synthetic_segments(N, T, seed=7, device=dev, coef=F4, dt=0.1)
V = coh.x[:T, :N].t().contiguous()
arm = coh.arm[:, :N].t().contiguous()
g = torch.Generator(device=dev)
g.manual_seed(N)
sl = torch.randint(1, T + 1, (N,), generator=g, device=dev, dtype=torch.int32)
base = np.array(F4) * 1.1
c0 = np.where(base != 0, base, 0.01)
nf = torch.empty((N,), dtype=torch.int32, device=dev)
for rep in range(int(os.environ.get("PROF_REPS", 3))):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r = ops.insite_refine(V, arm, coh.u, sl, c0, coh.lib, coh.dt, 10.0, 5, nfev=nf)
    e1.record()
    torch.cuda.synchronize()
    print(f"call {rep}: {e0.elapsed_time(e1):.3f} ms, mean nfev {nf.double().mean().item():.3f}", flush=True)
