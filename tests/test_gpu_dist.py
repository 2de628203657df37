"""GPU: the multi-rank discovery path on device, rehearsed with 2 ranks on ONE GPU
over gloo (the driver's 8-GPU runs use RCCL; same code with the backend swapped).

Each rank runs the product path on its contiguous patient shard — the Gram kernel into a MomentBuffer
(insite_gram_f64), ONE all-reduce of the packed G|b (or the deterministic all-gather + rank-ordered
sum), then the replicated STLSQ kernel (insite_stlsq_f64) — and the masked-SSE metric sums of its
shard (insite_masked_sse_f64) reduced in one collective.  Both must equal the single-rank fused fit
and metrics on the whole cohort: identical support, coefficient L-inf < 1e-12, identical models on
both ranks, the deterministic reduction bitwise equal on both ranks.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd")
N, T = 20_000, 60


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cohort(dev):
    from insite_amd import cohort
    return cohort.synthetic_pkpd(N, T, seed=4242, device=dev, equation="EQ_4_C")


def _metric_inputs(coh, dev):
    g = torch.Generator(device=dev)
    g.manual_seed(99)
    pred = coh.x[:, :T] + 0.01 * torch.randn((N, T), generator=g, device=dev, dtype=torch.float64)
    sl = torch.randint(2, T + 1, (N,), generator=g, device=dev)
    active = (torch.arange(T, device=dev)[None, :] < sl[:, None]).to(torch.float64)
    return pred.contiguous(), coh.x[:, :T].contiguous(), active.contiguous()


def _worker(rank, world, port, q):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from insite_amd import dist as idist
    from insite_amd import ops
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        coh = _cohort(dev)
        lo, hi = idist.shard_bounds(N, rank, world)
        sl = slice(lo, hi)
        res = {}
        for det in (False, True):
            buf = idist.MomentBuffer(2, coh.lib.n_terms, dev)
            coef, mask, _ = idist.discover_sharded(coh.x[sl], coh.u[sl].contiguous(), coh.arm[sl].contiguous(),
                                                   coh.rows[sl].contiguous(), coh.dt, coh.lib, 0.1, 0.5, buf,
                                                   deterministic=det)
            torch.cuda.synchronize()
            res[det] = (coef.cpu().numpy(), mask.cpu().numpy(), buf.flat.cpu().numpy())
        pred, tgt, act = _metric_inputs(coh, dev)
        per, cnt, last = ops.masked_sse(pred[sl], tgt[sl].contiguous(), act[sl].contiguous())
        per, cnt, last = idist.reduce_metric_sums(per, cnt, last)
        met = idist.rmse_from_sums(per, cnt, last)
        q.put((rank, res, met))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_two_rank_discovery_and_metrics_equal_single_rank(dev):
    from insite_amd import ops
    from insite_amd import dist as idist
    coh = _cohort(dev)
    coef, mask, _, G, b = ops.sindy_fit(coh.x, coh.u, coh.arm, coh.rows, coh.dt, coh.lib, 0.1, 0.5)
    pred, tgt, act = _metric_inputs(coh, dev)
    ref_met = idist.rmse_from_sums(*ops.masked_sse(pred, tgt, act))
    torch.cuda.synchronize()
    coef, mask = coef.cpu().numpy(), mask.cpu().numpy()
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=180) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, res, met in out:
        for det in (False, True):
            c, m, _ = res[det]
            assert np.array_equal(m != 0, mask != 0)
            assert np.max(np.abs(c - coef)) < 1e-12
        np.testing.assert_allclose(met, ref_met, rtol=1e-12)
    # replicated STLSQ: identical models on both ranks; the rank-ordered sum is bitwise identical too
    for det in (False, True):
        np.testing.assert_array_equal(out[0][1][det][0], out[1][1][det][0])
    np.testing.assert_array_equal(out[0][1][True][2], out[1][1][True][2])
