#!/usr/bin/env python3
"""Achievable HBM bandwidth on this box: write-only (fill), read-only (sum) and
copy over 4 GB buffers, timed with HIP events.  Reported beside the rollout's roofline."""
import json
import torch

dev = torch.device("cuda:0")
n = 4_000_000_000 // 8
a = torch.empty(n, dtype=torch.float64, device=dev)
b = torch.empty(n // 2, dtype=torch.float64, device=dev)
c = torch.empty(n // 2, dtype=torch.float64, device=dev)


def timed(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


out = {}
t = timed(lambda: a.fill_(1.0))
out["write_TBps"] = a.numel() * 8 / t / 1e12
t = timed(lambda: a.sum())
out["read_TBps"] = a.numel() * 8 / t / 1e12
t = timed(lambda: c.copy_(b))
out["copy_TBps_rw"] = 2 * b.numel() * 8 / t / 1e12
print(json.dumps(out))
