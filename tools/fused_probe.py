"""Fused step kernel probe: each role alone vs its block count (the other role given a token cohort),
to see how the discovery and the rollout scale with waves at the step kernel's 2-waves/SIMD budget."""
import os
import sys
import json

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd"))
import torch  # noqa: E402
from insite_amd import ops, cohort  # noqa: E402

dev = torch.device("cuda:0")
N, T = 100_000, 200
big = cohort.synthetic_pkpd(N, T, seed=1, device=dev, equation="EQ_4_C", layout="time")
tiny = cohort.synthetic_pkpd(64, T, seed=2, device=dev, equation="EQ_4_C", layout="time")
bits_big = cohort.counterfactual_arms(big.arm, T, seed=3, layout="time_bits")
bits_tiny = cohort.counterfactual_arms(tiny.arm, T, seed=3, layout="time_bits")
lib = big.lib
cin = torch.zeros((2, lib.n_terms), dtype=torch.float64, device=dev)
cin[0, 4], cin[1, 1], cin[1, 5] = -1.11, -0.145, -1.02
y = torch.empty((T, N), dtype=torch.float64, device=dev)


def timeit(fn, n=30):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


res = {}
for gb in [int(v) for v in os.environ.get("GBS", "64 128 192 256 320 384 448").split()]:
    # rollout alone on 512 - gb blocks (the discovery of 64 patients on gb blocks)
    pr = ops.plan_fit_rollout(tiny.x, tiny.u, tiny.arm, tiny.rows, tiny.dt, lib, 0.1, 0.5, big.y0, big.u, bits_big,
                              cin, big.dt, method="rk4", T=T, y_out=y, gram_blocks=gb)
    # discovery alone on gb blocks (a 64-patient rollout)
    yt = torch.empty((T, 64), dtype=torch.float64, device=dev)
    pg = ops.plan_fit_rollout(big.x, big.u, big.arm, big.rows, big.dt, lib, 0.1, 0.5, tiny.y0, tiny.u, bits_tiny,
                              cin, tiny.dt, method="rk4", T=T, y_out=yt, gram_blocks=gb)
    res[gb] = {"rollout_only_us": timeit(pr), "discovery_only_us": timeit(pg)}
    print(gb, {k: round(v, 2) for k, v in res[gb].items()}, flush=True)
rp = ops.plan_rollout(big.y0, big.u, bits_big, cin, lib, big.dt, method="rk4", T=T, out=y, layout="time_bits")
gp = ops.plan_sindy_fit(big.x, big.u, big.arm, big.rows, big.dt, lib, 0.1, 0.5, layout="time")
print("standalone rollout_us", round(timeit(rp), 2), "standalone discovery_us", round(timeit(gp), 2))
