"""Multi-process (gloo, world_size 2, CPU) tests of the sharded discovery path.

The GPU path (insite_amd.dist.discover_sharded) is: per-rank Gram over a contiguous patient
shard -> ONE all-reduce(SUM) of the packed G|b buffer -> replicated STLSQ.  Here each rank builds
its shard's partial moments with the oracle (the Gram kernel's CPU restatement), and the product
host logic (shard_bounds, MomentBuffer packing, reduce_moments, max_over_ranks) runs unchanged
over gloo.  The reduced system must equal the single-process full-cohort one, and the STLSQ on
it must give the same model on every rank.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    from oracle import insite_ref as R
    from insite_amd import dist as idist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        g = np.load(os.path.join(ROOT, "tests", "golden", "discovery_eq_4_c.npz"))
        x, u, arm, rows = g["x"], g["u"], g["arm"], g["rows"]
        lo, hi = idist.shard_bounds(x.shape[0], rank, world)
        exps = R.poly_library(3, 2, True)
        buf = idist.MomentBuffer(2, exps.shape[0], "cpu")
        G, b = R.gram_moments(x[lo:hi], u[lo:hi], arm[lo:hi], rows[lo:hi], float(g["dt"]), exps)
        buf.G.copy_(torch.from_numpy(G))
        buf.b.copy_(torch.from_numpy(b))
        idist.reduce_moments(buf)
        coefs = [R.stlsq_gram(buf.G[a].numpy(), buf.b[a].numpy(), 0.1, 0.5)[0] for a in range(2)]
        t = idist.max_over_ranks(0.5 + rank)
        q.put((rank, lo, hi, buf.flat.numpy().copy(), np.stack(coefs), t))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_shard_bounds_partition():
    from insite_amd.dist import shard_bounds
    for n in (0, 1, 7, 100, 100_003):
        for w in (1, 2, 3, 8):
            spans = [shard_bounds(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [h - l_ for l_, h in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_bounds(10, 2, 2)


def test_moment_buffer_views():
    from insite_amd.dist import MomentBuffer
    m = MomentBuffer(2, 7, "cpu")
    assert m.flat.numel() == 2 * 49 + 14
    m.G[1, 2, 3] = 5.0
    m.b[0, 6] = 7.0
    assert m.flat[49 + 2 * 7 + 3] == 5.0 and m.flat[98 + 6] == 7.0


def test_sharded_discovery_gloo_world2():
    from oracle import insite_ref as R
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    g = np.load(os.path.join(ROOT, "tests", "golden", "discovery_eq_4_c.npz"))
    # shards tile the cohort
    assert res[0][1] == 0 and res[0][2] == res[1][1] and res[1][2] == g["x"].shape[0]
    full = np.concatenate([g["G"].reshape(-1), g["b"].reshape(-1)])
    for r in res:
        np.testing.assert_allclose(r[3], full, rtol=1e-12, atol=1e-9)   # all-reduced == full cohort
        assert r[5] == 1.5                                              # max over ranks
    np.testing.assert_array_equal(res[0][4], res[1][4])                 # replicated STLSQ identical
    assert np.max(np.abs(res[0][4] - g["coef"])) < 1e-8
    assert np.array_equal(res[0][4] != 0, g["mask"].astype(bool))


def _metric_worker(rank, world, port, q):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    from oracle import insite_ref as R
    from insite_amd import dist as idist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        g = np.load(os.path.join(ROOT, "tests", "golden", "metrics.npz"))
        pred, target, active = g["pred"][..., 0], g["target"][..., 0], g["active"][..., 0]
        lo, hi = idist.shard_bounds(pred.shape[0], rank, world)
        err = (pred[lo:hi] - target[lo:hi]) ** 2 * active[lo:hi]
        nxt = np.concatenate([active[lo:hi, 1:], np.zeros((hi - lo, 1))], axis=1)
        lastm = active[lo:hi] - nxt                              # the final active entry of each row
        per = torch.from_numpy(err.sum(0))
        cnt = torch.from_numpy(active[lo:hi].sum(0))
        last = torch.tensor([(err * lastm).sum(), lastm.sum()], dtype=torch.float64)
        red = idist.reduce_metric_sums(per, cnt, last)
        det = idist.reduce_metric_sums(per, cnt, last, deterministic=True)
        x = torch.full((5,), 0.1 * (rank + 1), dtype=torch.float64)
        idist.fixed_order_sum(x)
        q.put((rank, idist.rmse_from_sums(*red), idist.rmse_from_sums(*det), x.numpy().copy()))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_metric_sums_all_reduce_gloo_world3():
    """each rank's masked (SSE, count) partial sums, reduced in one collective (all-reduce
    or the deterministic rank-ordered all-gather sum), give the full-cohort RMSE metrics (golden
    fixture tests/golden/metrics.npz); the fixed-order sum equals the rank-ordered CPU sum bitwise."""
    world = 3
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_metric_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = np.load(os.path.join(ROOT, "tests", "golden", "metrics.npz"))
    want = [float(g["rmse_orig"]), float(g["rmse_all"]), float(g["rmse_last"])]
    for _, red, det, x in res:
        np.testing.assert_allclose(red, want, rtol=1e-12)
        np.testing.assert_allclose(det, want, rtol=1e-12)
        assert np.array_equal(x, np.full(5, (0.1 + 0.2) + 0.3))


def _bucket_worker(rank, world, port, q):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    from insite_amd import dist as idist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        bk = idist.MomentBucket(4, 2, 7, "cpu")
        for k, buf in enumerate(bk.bufs):   # every fit's partial: distinct per (rank, step)
            buf.G.copy_(torch.full((2, 7, 7), 10.0 * k + rank))
            buf.b.copy_(torch.full((2, 7), -(10.0 * k + rank)))
        idist.reduce_bucket(bk)
        q.put((rank, [(b.G.clone().numpy(), b.b.clone().numpy()) for b in bk.bufs]))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def test_bucketed_allreduce_reduces_every_fit_in_one_collective():
    """The C2 pipeline's N > 1 batching: K fits' G|b views of one flat buffer, one all-reduce (gloo, 2
    ranks): every view holds the sum over ranks of its own fit's partial."""
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        for k, (G, b) in enumerate(res[r]):
            want = sum(10.0 * k + rr for rr in range(world))
            assert np.all(G == want) and np.all(b == -want)



def _lagged_worker(rank, world, port, q, K, n_launch, delay=0):
    """Each rank plays insite_fit_rollout_lagged_f64's roles with the oracle's CPU restatements on its own
    shard: the gram (slot write), the block reduction (slot -> bucket entry), the replicated STLSQ (bucket
    entry -> coefficient ring) and the rollout (ring -> y), in exactly the order LaggedSchedule gives, with the
    bucket all-reduce (gloo) after the launches it names -- with delay 1 issued async and waited for only before
    the launch whose solve first reads the bucket (``wait_before``)."""
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    from oracle import insite_ref as R
    from insite_amd import dist as idist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        g = np.load(os.path.join(ROOT, "tests", "golden", "discovery_eq_4_c.npz"))
        x, u, arm, rows = g["x"], g["u"], g["arm"], g["rows"]
        lo, hi = idist.shard_bounds(x.shape[0], rank, world)
        exps = R.poly_library(3, 2, True)
        F = exps.shape[0]

        def cohort_x(c):   # cohort c: the golden cohort rescaled per c (distinct systems per launch)
            return x * (1.0 + 0.01 * c)

        sched = idist.LaggedSchedule(K, delay)
        slots = [None, None]
        buckets = [idist.MomentBucket(K, 2, F, "cpu") for _ in range(sched.NB)]
        handles = {}
        ring = [None] * 3
        fitted, rolled = {}, {}
        for k in range(n_launch):
            p = sched.launch(k)
            if p["wait_before"] is not None:
                handles.pop(p["wait_before"]).wait()
            # roles read state as the kernel does: the gram writes slot k % 2, the reduction reads the other
            cur = R.gram_moments(cohort_x(k)[lo:hi], u[lo:hi], arm[lo:hi], rows[lo:hi], float(g["dt"]), exps)
            if p["reduce"] is not None:
                c, bi, pos = p["reduce"]
                G, b = slots[(k - 1) % 2]
                buckets[bi].bufs[pos].G.copy_(torch.from_numpy(G))
                buckets[bi].bufs[pos].b.copy_(torch.from_numpy(b))
            if p["fit"] is not None:
                c, bi, pos, r = p["fit"]
                buf = buckets[bi].bufs[pos]
                ring[r] = (c, np.stack([R.stlsq_gram(buf.G[a].numpy(), buf.b[a].numpy(), 0.1, 0.5)[0]
                                        for a in range(2)]))
                fitted[c] = ring[r][1]
            if p["rollout"] is not None:
                c, r = p["rollout"]
                assert ring[r][0] == c        # the rollout reads ITS cohort's model
                rolled[c] = ring[r][1]
            slots[k % 2] = cur
            if p["allreduce_after"] is not None:
                if delay:
                    handles[p["allreduce_after"]] = idist.reduce_bucket(buckets[p["allreduce_after"]], async_op=True)
                else:
                    idist.reduce_bucket(buckets[p["allreduce_after"]])
        for h in handles.values():
            h.wait()
        q.put((rank, fitted, rolled))
    finally:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.parametrize("K,delay", [(1, 0), (4, 0), (1, 1), (4, 1)])
def test_lagged_schedule_gloo_world2(K, delay):
    """The N > 1 lagged step's bookkeeping (insite_amd.dist.LaggedSchedule; bench.py lagged_run) over gloo with 2
    ranks: every cohort's model is the STLSQ of the ALL-RANK Gram (equal to a single-process fit of the whole
    cohort), identical on both ranks, and every rollout uses its own cohort's model."""
    from oracle import insite_ref as R
    world, n_launch = 2, 4 * K + 8
    L = (1 + delay) * K
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_lagged_worker, args=(r, world, port, q, K, n_launch, delay)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (f, ro) for r, f, ro in (q.get(timeout=180) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = np.load(os.path.join(ROOT, "tests", "golden", "discovery_eq_4_c.npz"))
    exps = R.poly_library(3, 2, True)
    fitted0, rolled0 = res[0]
    assert sorted(fitted0) == list(range(n_launch - L - 1))
    assert sorted(rolled0) == list(range(n_launch - L - 2))
    for c, coef in fitted0.items():
        G, b = R.gram_moments(g["x"] * (1.0 + 0.01 * c), g["u"], g["arm"], g["rows"], float(g["dt"]), exps)
        want = np.stack([R.stlsq_gram(G[a], b[a], 0.1, 0.5)[0] for a in range(2)])
        assert np.array_equal(coef != 0, want != 0)
        np.testing.assert_allclose(coef, want, rtol=1e-9, atol=1e-12)
        assert np.array_equal(coef, res[1][0][c])      # replicated solve: bitwise on both ranks
    for c, coef in rolled0.items():
        assert np.array_equal(coef, fitted0[c])


def test_lagged_schedule_never_aliases():
    """Within one launch the solve never reads the bucket entry the reduction writes, the all-reduced bucket
    is complete (its K cohorts reduced) and not yet rewritten when its fits read it, and the rollout's ring slot
    is never the one the solve writes."""
    from insite_amd.dist import LaggedSchedule
    for K, D in [(K, D) for K in (1, 2, 4, 8) for D in (0, 1)]:
        s = LaggedSchedule(K, D)
        reduced_at, allreduced_at, waited_at = {}, {}, {}
        writes = {}
        for k in range(20 * K + 10):
            p = s.launch(k)
            if p["wait_before"] is not None:                # delay 1: waited for K launches after its issue
                j = next(jj for jj in allreduced_at if jj % s.NB == p["wait_before"] and jj not in waited_at)
                assert k - allreduced_at[j] >= K
                waited_at[j] = k
            if p["reduce"]:
                c, bi, pos = p["reduce"]
                reduced_at[c] = k
                writes[(bi, pos)] = c
            if p["fit"]:
                c, bi, pos, r = p["fit"]
                assert writes[(bi, pos)] == c                       # entry still holds cohort c
                assert not p["reduce"] or p["reduce"][1] != bi      # not the bucket being written
                assert allreduced_at.get(c // K, 10 ** 9) < k        # its bucket was all-reduced before
                assert not D or waited_at.get(c // K, 10 ** 9) <= k   # ... and waited for (delay 1)
                assert not p["rollout"] or p["rollout"][1] != r
            if p["allreduce_after"] is not None:
                j = (k - 1) // K
                assert all(reduced_at.get(c, 10 ** 9) <= k for c in range(j * K, j * K + K))
                allreduced_at[j] = k
