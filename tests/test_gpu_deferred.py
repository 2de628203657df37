"""The C2 bench's own kernels against the ORACLE at the bench's configuration ("RMSE vs CPU ref").

* ``insite_fit_rollout_deferred_f64`` (step_deferred_kernel, the timed N = 1 launch) on the bench's own 100k x
  200 cohort (cohort.synthetic_pkpd seed 1000 = bench.py --seed 1, rank 0): the model finalised by the stream
  equals the oracle's SINDy fit of that cohort (support identical, coefficient L-inf < 1e-8) and the rollout the
  next launch writes with it equals the oracle's RK4 scan on sampled rows (rtol 1e-10, RMSE < 1e-6) --
  oracle/insite_ref.py restates sindy.py:190-192 (fit) and :371-431 (scan).
* The slot record (ABI 8): consecutive calls that change the method (and so the default block split) still
  finalise the right number of partials; a slot no call has streamed is flagged (iters -3, NaN), not summed.
* ``insite_fit_rollout_lagged_f64`` (the N > 1 step): its reduction role writes the same G|b as the deferred
  finalisation, its solve role the same coefficients from a given G|b, and a LaggedSchedule stream with K = 2
  on one rank (the all-reduce of a single rank is the identity) reproduces the deferred stream's models and
  trajectories bitwise.
"""
import numpy as np
import pytest
import torch

from oracle import insite_ref as R

pytestmark = pytest.mark.gpu

N, T = 100_000, 200


@pytest.fixture(scope="module")
def bench_cohort(dev):
    from insite_amd import cohort
    coh = cohort.synthetic_pkpd(N, T, seed=1000, device=dev, equation="EQ_4_C", layout="time")
    bits = cohort.counterfactual_arms(coh.arm, T, seed=1000, layout="time_bits")
    return coh, bits


def _outs(dev, F):
    return (torch.zeros((2, F), dtype=torch.float64, device=dev), torch.zeros((2, F), dtype=torch.int8, device=dev),
            torch.zeros((2,), dtype=torch.int32, device=dev), torch.zeros((2, F, F), dtype=torch.float64, device=dev),
            torch.zeros((2, F), dtype=torch.float64, device=dev))


def _oracle_model(coh):
    x = coh.x[:, :N].t().contiguous().cpu().numpy()
    u, arm = coh.u.cpu().numpy(), coh.arm.cpu().numpy().astype(np.int64)
    exps = coh.lib.exps.astype(np.int64)
    G, b = R.gram_moments_vectorized(x, u, arm, T - 2, coh.dt, exps)
    return G, b, np.stack([R.stlsq_gram(G[a], b[a], 0.1, 0.5)[0] for a in range(2)])


def _sample_rows(dev, coh, bits, coef_np, y, n=4000, seed=3):
    rng = np.random.default_rng(seed)
    idx = np.unique(np.concatenate([rng.choice(N, n, replace=False), np.arange(64), np.arange(N - 96, N)]))
    it = torch.as_tensor(idx, device=dev)
    words = bits.index_select(1, it // 32)
    arms = ((words >> (it % 32).to(torch.int32)[None, :]) & 1).t().contiguous().cpu().numpy().astype(np.int64)
    ref = R.rollout(coh.y0[it].cpu().numpy(), coh.u[it].cpu().numpy(), arms, coef_np,
                    coh.lib.exps.astype(np.int64), coh.dt, method="rk4")
    return y.index_select(1, it).t().cpu().numpy(), ref


def test_deferred_step_on_bench_cohort_matches_oracle(dev, bench_cohort):
    from insite_amd import ops
    coh, bits = bench_cohort
    lib = coh.lib
    F = lib.n_terms
    ws = ops.Workspace()
    o = [_outs(dev, F) for _ in range(3)]
    y = torch.empty((T, N), dtype=torch.float64, device=dev)
    # the bench's stream on one cohort: call 0 streams slot 0; call 1 finalises it into o[1]; call 2 rolls the
    # cohort out with o[1] (the model of the same cohort) while finalising call 1's slot into o[2]
    for k in range(3):
        ops.fit_rollout_deferred(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, coh.y0, coh.u, bits,
                                 o[(k - 1) % 3][0], coh.dt, k % 2, k > 0, ws, method="rk4", T=T, y_out=y,
                                 out=o[k % 3] if k > 0 else o[2])
    torch.cuda.synchronize()
    G, b, cr = _oracle_model(coh)
    for j in (1, 2):   # both finalisations of the same cohort
        coef, mask, iters, Gg, bg = (t.cpu().numpy() for t in o[j])
        np.testing.assert_allclose(Gg, G, rtol=1e-10, atol=1e-6)
        np.testing.assert_allclose(bg, b, rtol=1e-10, atol=1e-6)
        assert np.array_equal(mask != 0, cr != 0)
        assert np.max(np.abs(coef - cr)) < 1e-8
        assert np.all(iters > 0)
    got, ref = _sample_rows(dev, coh, bits, cr, y)
    np.testing.assert_allclose(got, ref, rtol=1e-10)
    assert np.sqrt(np.mean((got - ref) ** 2)) < 1e-6


def test_deferred_slot_record_survives_method_change(dev, bench_cohort):
    """the finalisation must sum the partial count the STREAMING call used.  rk4 and euler5 launches
    have different default gram block counts; alternating them must still give G|b of a plain fit (rtol 1e-12)."""
    from insite_amd import ops
    coh, bits = bench_cohort
    lib = coh.lib
    F = lib.n_terms
    ws = ops.Workspace()
    o = [_outs(dev, F) for _ in range(2)]
    y = torch.empty((T, N), dtype=torch.float64, device=dev)
    cin = torch.zeros((2, F), dtype=torch.float64, device=dev)
    for k, meth, gblk in ((0, "rk4", 0), (1, "euler5", 0), (2, "rk4", 77), (3, "euler5", 0)):
        ops.fit_rollout_deferred(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, coh.y0, coh.u, bits, cin,
                                 coh.dt, k % 2, k > 0, ws, method=meth, T=T, y_out=y, out=o[k % 2],
                                 gram_blocks=gblk)
        if k > 0:
            torch.cuda.synchronize()
            c2, m2, _, G2, b2 = ops.sindy_fit(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, layout="time")
            np.testing.assert_allclose(o[k % 2][3].cpu().numpy(), G2.cpu().numpy(), rtol=1e-12, atol=1e-9)
            np.testing.assert_allclose(o[k % 2][4].cpu().numpy(), b2.cpu().numpy(), rtol=1e-12, atol=1e-9)
            assert torch.equal(o[k % 2][1], m2)


def test_deferred_unstreamed_slot_is_flagged(dev):
    from insite_amd import cohort, ops
    coh = cohort.synthetic_pkpd(3000, 40, seed=3, device=dev, equation="EQ_4_C", layout="time")
    bits = cohort.counterfactual_arms(coh.arm, 40, seed=3, layout="time_bits")
    F = coh.lib.n_terms
    ws = ops.Workspace()
    ws.claim("deferred").get(1 << 22, dev).fill_(0x5A)          # garbage headers: no call streamed slot 1
    out = _outs(dev, F)
    ops.fit_rollout_deferred(coh.x, coh.u, coh.arm, coh.rows, coh.dt, coh.lib, 0.1, 0.5, coh.y0, coh.u, bits,
                             torch.zeros((2, F), dtype=torch.float64, device=dev), coh.dt, 0, True, ws, T=40, out=out)
    torch.cuda.synchronize()
    coef, mask, iters, G, b = out
    assert torch.all(iters == -3) and torch.isnan(coef).all() and torch.isnan(G).all() and not mask.any()


def test_deferred_slot_streamed_for_another_system_is_flagged(dev):
    """A slot streamed with one 7-term library and finalised by a call with another of the same shape (the same
    columns in another order: same F, arm count and statics) is flagged through the slot record's fingerprint, not
    summed as this library's G|b; the same library finalises normally."""
    from insite_amd import cohort, ops
    from insite_amd.library import PolyLibrary
    coh = cohort.synthetic_pkpd(3000, 40, seed=3, device=dev, equation="EQ_4_C", layout="time")
    bits = cohort.counterfactual_arms(coh.arm, 40, seed=3, layout="time_bits")
    F = coh.lib.n_terms
    other = PolyLibrary(np.ascontiguousarray(coh.lib.exps[::-1]), coh.lib.input_names, coh.lib.n_inputs)
    cin = torch.zeros((2, F), dtype=torch.float64, device=dev)
    for lib2, flagged in ((other, True), (coh.lib, False)):
        ws = ops.Workspace()
        out = [_outs(dev, F) for _ in range(2)]
        ops.fit_rollout_deferred(coh.x, coh.u, coh.arm, coh.rows, coh.dt, coh.lib, 0.1, 0.5, coh.y0, coh.u, bits, cin,
                                 coh.dt, 0, False, ws, T=40, out=out[0])
        ops.fit_rollout_deferred(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib2, 0.1, 0.5, coh.y0, coh.u, bits, cin,
                                 coh.dt, 1, True, ws, T=40, out=out[1])
        torch.cuda.synchronize()
        coef, mask, iters, G, b = out[1]
        if flagged:
            assert torch.all(iters == -3) and torch.isnan(coef).all() and torch.isnan(G).all() and not mask.any()
        else:
            assert torch.all(iters >= 0) and torch.isfinite(G).all()


def test_lagged_roles_equal_deferred(dev, bench_cohort):
    """Reduction role == the deferred finalisation's G|b (bitwise: same partials, same association); solve role
    == the deferred STLSQ on that G|b (bitwise); rollout == the deferred rollout (bitwise)."""
    from insite_amd import ops
    coh, bits = bench_cohort
    lib = coh.lib
    F = lib.n_terms
    cin = torch.zeros((2, F), dtype=torch.float64, device=dev)
    cin[0, 4], cin[1, 1], cin[1, 5] = -1.1107592869834308, -0.14540553723951796, -1.0234639833519243
    # deferred reference: two calls
    wsd = ops.Workspace()
    od = _outs(dev, F)
    yd = torch.empty((T, N), dtype=torch.float64, device=dev)
    for k in range(2):
        ops.fit_rollout_deferred(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, coh.y0, coh.u, bits, cin,
                                 coh.dt, k, k > 0, wsd, T=T, y_out=yd, out=od)
    # lagged: call 0 streams; call 1 reduces into (Gr, br) and solves the deferred G|b given as G_fit
    wsl = ops.Workspace()
    Gr = torch.zeros((2, F, F), dtype=torch.float64, device=dev)
    br = torch.zeros((2, F), dtype=torch.float64, device=dev)
    fit = (torch.zeros((2, F), dtype=torch.float64, device=dev), torch.zeros((2, F), dtype=torch.int8, device=dev),
           torch.zeros((2,), dtype=torch.int32, device=dev))
    yl = torch.empty((T, N), dtype=torch.float64, device=dev)
    for k in range(2):
        p = ops.plan_fit_rollout_lagged(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, coh.y0, coh.u, bits,
                                        cin, coh.dt, k, k > 0, wsl, (Gr, br),
                                        fit_in=(od[3], od[4]) if k > 0 else None, fit_out=fit if k > 0 else None,
                                        T=T, y_out=yl)
        p()
    torch.cuda.synchronize()
    assert torch.equal(Gr, od[3]) and torch.equal(br, od[4])
    assert torch.equal(fit[0], od[0]) and torch.equal(fit[1], od[1]) and torch.equal(fit[2], od[2])
    assert torch.equal(yl, yd)


def test_lagged_stream_single_rank_matches_oracle(dev):
    """A LaggedSchedule stream (K = 2, two rotating cohorts, the bench's lagged_run bookkeeping) on one rank:
    every solved model equals the oracle fit of its cohort and every rollout uses its own cohort's model."""
    from insite_amd import cohort, ops
    from insite_amd.dist import LaggedSchedule, MomentBucket
    n, t, K = 20_000, 80, 2
    cohs = [cohort.synthetic_pkpd(n, t, seed=77 + j, device=dev, equation="EQ_4_C", layout="time") for j in range(2)]
    bitss = [cohort.counterfactual_arms(c.arm, t, seed=77 + j, layout="time_bits") for j, c in enumerate(cohs)]
    lib = cohs[0].lib
    F = lib.n_terms
    sched = LaggedSchedule(K)
    buckets = [MomentBucket(K, 2, F, dev) for _ in range(2)]
    ring = [(torch.zeros((2, F), dtype=torch.float64, device=dev), torch.zeros((2, F), dtype=torch.int8, device=dev),
             torch.zeros((2,), dtype=torch.int32, device=dev)) for _ in range(3)]
    ys = [torch.empty((t, n), dtype=torch.float64, device=dev) for _ in range(2)]
    ws = ops.Workspace()
    dummy = torch.zeros((2, F), dtype=torch.float64, device=dev)
    Gs, bs = torch.zeros((2, F, F), dtype=torch.float64, device=dev), torch.zeros((2, F), dtype=torch.float64,
                                                                                   device=dev)
    solved, rolled = {}, {}
    for k in range(2 * K + 6):
        p = sched.launch(k)
        c = cohs[k % 2]
        red = (buckets[p["reduce"][1]].bufs[p["reduce"][2]].G, buckets[p["reduce"][1]].bufs[p["reduce"][2]].b) \
            if p["reduce"] else (Gs, bs)
        fit_in = fit_out = None
        if p["fit"]:
            fc, bi, pos, r = p["fit"]
            fit_in = (buckets[bi].bufs[pos].G, buckets[bi].bufs[pos].b)
            fit_out = ring[r]
        if p["rollout"]:
            rc_, r = p["rollout"]
            rcoh, rbits, coef_in, yy = cohs[rc_ % 2], bitss[rc_ % 2], ring[r][0], ys[rc_ % 2]
        else:
            rcoh, rbits, coef_in, yy = c, bitss[k % 2], dummy, ys[k % 2]
        ops.plan_fit_rollout_lagged(c.x, c.u, c.arm, c.rows, c.dt, lib, 0.1, 0.5, rcoh.y0, rcoh.u, rbits, coef_in,
                                    rcoh.dt, p["slot"], p["reduce"] is not None, ws, red, fit_in=fit_in,
                                    fit_out=fit_out, T=t, y_out=yy)()
        torch.cuda.synchronize()
        if p["fit"]:
            solved[p["fit"][0]] = ring[p["fit"][3]][0].cpu().numpy().copy()
        if p["rollout"]:
            rolled[p["rollout"][0]] = (ring[p["rollout"][1]][0].cpu().numpy().copy(), yy.clone())
        # (single rank: the all-reduce after launch k is the identity)
    want = []
    for j in range(2):
        x = cohs[j].x[:, :n].t().contiguous().cpu().numpy()
        G, b = R.gram_moments_vectorized(x, cohs[j].u.cpu().numpy(), cohs[j].arm.cpu().numpy().astype(np.int64),
                                         t - 2, cohs[j].dt, lib.exps.astype(np.int64))
        want.append(np.stack([R.stlsq_gram(G[a], b[a], 0.1, 0.5)[0] for a in range(2)]))
    assert sorted(solved) == list(range(2 * K + 6 - K - 1))
    for cc, coef in solved.items():
        assert np.array_equal(coef != 0, want[cc % 2] != 0)
        assert np.max(np.abs(coef - want[cc % 2])) < 1e-8
    for cc, (coef, yy) in rolled.items():
        assert np.array_equal(coef, solved[cc])
        y2 = ops.rollout(cohs[cc % 2].y0, cohs[cc % 2].u, bitss[cc % 2], torch.as_tensor(coef, device=dev), lib,
                         cohs[cc % 2].dt, method="rk4", T=t, layout="time_bits")
        assert torch.equal(yy, y2)


def _ns_gram_job(job):
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    from oracle import insite_ref as Q
    return Q.gram_moments_vectorized(*job)


def test_deferred_step_north_star_1m_x_500_matches_oracle(dev):
    """BASELINE.json north_star's configuration (1M patients x 500 steps, fp64) through the timed N = 1 kernel, as the
    default bench line's ``north_star_step`` block runs it (cohort seed 1900 = bench.py --seed 1): the finalised model
    against the oracle's SINDy fit of the WHOLE cohort (the oracle Gram in 32 patient chunks on a spawned pool, summed
    in chunk order; G|b rtol 1e-10, support identical, coefficient L-inf < 1e-8 -- north_star's bar) and the rollout
    the next launch writes with it against the oracle's RK4 scan on sampled rows (rtol 1e-10, RMSE < 1e-6)."""
    import multiprocessing as mp
    import os
    from insite_amd import cohort, ops
    Nn, Tn = 1_000_000, 500
    coh = cohort.synthetic_pkpd(Nn, Tn, seed=1900, device=dev, equation="EQ_4_C", layout="time")
    bits = cohort.counterfactual_arms(coh.arm, Tn, seed=1900, layout="time_bits")
    lib = coh.lib
    F = lib.n_terms
    ws = ops.Workspace()
    o = [_outs(dev, F) for _ in range(3)]
    y = torch.empty((Tn, Nn), dtype=torch.float64, device=dev)
    for k in range(3):
        ops.fit_rollout_deferred(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, coh.y0, coh.u, bits,
                                 o[(k - 1) % 3][0], coh.dt, k % 2, k > 0, ws, method="rk4", T=Tn, y_out=y,
                                 out=o[k % 3] if k > 0 else o[2])
    torch.cuda.synchronize()
    u, arm = coh.u.cpu().numpy(), coh.arm.cpu().numpy().astype(np.int64)
    exps = lib.exps.astype(np.int64)
    bounds = [(int(c[0]), int(c[-1]) + 1) for c in np.array_split(np.arange(Nn), 32)]
    jobs = [(coh.x[:, lo:hi].t().contiguous().cpu().numpy(), u[lo:hi], arm[lo:hi], Tn - 2, coh.dt, exps)
            for lo, hi in bounds]
    W = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS") or 8), os.cpu_count() or 1))
    with mp.get_context("spawn").Pool(W) as pool:
        parts = pool.map(_ns_gram_job, jobs)
    del jobs
    G, b = sum(q[0] for q in parts), sum(q[1] for q in parts)
    cr = np.stack([R.stlsq_gram(G[a], b[a], 0.1, 0.5)[0] for a in range(2)])
    for j in (1, 2):
        coef, mask, iters, Gg, bg = (t.cpu().numpy() for t in o[j])
        np.testing.assert_allclose(Gg, G, rtol=1e-10, atol=1e-6)
        np.testing.assert_allclose(bg, b, rtol=1e-10, atol=1e-6)
        assert np.array_equal(mask != 0, cr != 0)
        assert np.max(np.abs(coef - cr)) < 1e-8
    rng = np.random.default_rng(5)
    idx = np.unique(np.concatenate([rng.choice(Nn, 3000, replace=False), np.arange(64), np.arange(Nn - 96, Nn)]))
    it = torch.as_tensor(idx, device=dev)
    words = bits.index_select(1, it // 32)
    arms = ((words >> (it % 32).to(torch.int32)[None, :]) & 1).t().contiguous().cpu().numpy().astype(np.int64)
    ref = R.rollout(coh.y0[it].cpu().numpy(), coh.u[it].cpu().numpy(), arms, cr, exps, coh.dt, method="rk4")
    got = y.index_select(1, it).t().cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-10)
    assert np.sqrt(np.mean((got - ref) ** 2)) < 1e-6


def test_claimed_gram_tail_stale_claim_area_is_flagged(dev):
    """The claimed gram tail (INSITE_DEF_DYN, taken where the gram waves stream >= 128 units each: this 300k x 460
    cohort, 136k units) keeps its per-XCD heads in the workspace's claim area, self-resetting.  A stale area (a head
    left on a value past its segment, as a reused buffer could hold) makes that launch skip the segment's pieces: the
    next finalisation of its slot must flag it (NaN G|b, iters -3), not sum a partial Gram, and the launch after it
    (the area reset by the stale launch's last wave) must finalise the right model again (G|b vs the static fit of the
    same cohort, rtol 1e-10)."""
    from insite_amd import cohort, ops
    Nn, Tn = 300_000, 460
    coh = cohort.synthetic_pkpd(Nn, Tn, seed=4242, device=dev, equation="EQ_4_C", layout="time")
    bits = cohort.counterfactual_arms(coh.arm, Tn, seed=4242, layout="time_bits")
    lib = coh.lib
    F = lib.n_terms
    ws = ops.Workspace()
    o = [_outs(dev, F) for _ in range(4)]
    y = torch.empty((Tn, Nn), dtype=torch.float64, device=dev)
    cin = torch.zeros((2, F), dtype=torch.float64, device=dev)

    def call(k, out):
        ops.fit_rollout_deferred(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, coh.y0, coh.u, bits, cin,
                                 coh.dt, k % 2, k > 0, ws, method="rk4", T=Tn, y_out=y, out=out)
    call(0, o[0])
    torch.cuda.synchronize()
    buf = next(iter(ws._buf.values()))
    buf[0:4] = torch.tensor([0xFF, 0xFF, 0xFF, 0x0F], dtype=torch.uint8, device=dev)   # head 0 stale
    call(1, o[1])          # streams slot 1 with the stale head; finalises slot 0 (clean)
    call(2, o[2])          # finalises slot 1: flagged
    call(3, o[3])          # finalises slot 0 (streamed by call 2 after the reset): clean
    torch.cuda.synchronize()
    ref = ops.sindy_fit(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, layout="time")
    torch.cuda.synchronize()
    Gr, br = ref[3].cpu().numpy(), ref[4].cpu().numpy()
    for j in (1, 3):
        np.testing.assert_allclose(o[j][3].cpu().numpy(), Gr, rtol=1e-10, atol=1e-6)
        np.testing.assert_allclose(o[j][4].cpu().numpy(), br, rtol=1e-10, atol=1e-6)
        assert np.array_equal(o[j][1].cpu().numpy(), ref[1].cpu().numpy())
    assert torch.isnan(o[2][3]).all() and torch.isnan(o[2][0]).all()
    assert (o[2][2] == -3).all()


def test_claimed_gram_tail_is_bitwise_reproducible_and_lagged_equal(dev):
    """The claimed gram tail's G|b do not depend on which wave took which piece (each piece's contribution has its own
    partial slot, summed in piece order): two independent deferred streams over the same 300k x 460 cohort (claimed
    instantiation; the claim order differs from run to run) finalise bitwise-equal G|b and models, and the lagged
    kernel's reduction role (the N > 1 step's dyn_finalize without the STLSQ) writes the same G|b bitwise."""
    from insite_amd import cohort, ops
    Nn, Tn = 300_000, 460
    coh = cohort.synthetic_pkpd(Nn, Tn, seed=4343, device=dev, equation="EQ_4_C", layout="time")
    bits = cohort.counterfactual_arms(coh.arm, Tn, seed=4343, layout="time_bits")
    lib = coh.lib
    F = lib.n_terms
    cin = torch.zeros((2, F), dtype=torch.float64, device=dev)
    y = torch.empty((Tn, Nn), dtype=torch.float64, device=dev)
    res = []
    for rep in range(2):
        ws = ops.Workspace()
        o = _outs(dev, F)
        for k in range(2):
            ops.fit_rollout_deferred(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, coh.y0, coh.u, bits, cin,
                                     coh.dt, k, k > 0, ws, T=Tn, y_out=y, out=o)
        torch.cuda.synchronize()
        res.append(tuple(t.clone() for t in o))
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)
    wsl = ops.Workspace()
    Gr = torch.zeros((2, F, F), dtype=torch.float64, device=dev)
    br = torch.zeros((2, F), dtype=torch.float64, device=dev)
    for k in range(2):
        ops.plan_fit_rollout_lagged(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, coh.y0, coh.u, bits, cin,
                                    coh.dt, k, k > 0, wsl, (Gr, br), T=Tn, y_out=y)()
    torch.cuda.synchronize()
    assert torch.equal(Gr, res[0][3]) and torch.equal(br, res[0][4])
    assert np.all(np.isfinite(Gr.cpu().numpy()))
