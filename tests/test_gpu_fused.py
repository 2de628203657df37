"""Fused step (insite_fit_rollout_f64, step_kernel): discovery of one cohort and the rollout of another
in one launch must give what the two separate calls give.

* rollout half: y bitwise equal to insite_rollout_f64 (time_bits) -- every rollout wave's range of
  (tile, arm group) units re-integrates its tile's earlier groups, so the stored states are the same
  FMA sequence from y0 (sizes with a partial last tile / last arm group, gram_blocks sweeping the split);
* discovery half: G/b to rtol 1e-12 of insite_sindy_fit_f64 (same fixed-order sums, a different block
  count), identical support, coefficient L-inf < 1e-10, and against the oracle (Gram rtol 1e-10,
  coefficients < 1e-8 -- the north-star tolerance);
* bitwise reproducible for a fixed split; gram-only call (n_rows = 0); unsupported shapes refused.
"""
import numpy as np
import pytest
import torch

from oracle import insite_ref as R

pytestmark = pytest.mark.gpu


def _cohorts(dev, N, T, Nr, Tr, seed=5):
    from insite_amd import cohort
    disc = cohort.synthetic_pkpd(N, T, seed=seed, device=dev, equation="EQ_4_C", layout="time")
    rc = cohort.synthetic_pkpd(Nr, Tr, seed=seed + 1, device=dev, equation="EQ_4_C", layout="time")
    bits = cohort.counterfactual_arms(rc.arm, Tr, seed=seed + 2, layout="time_bits")
    return disc, rc, bits


def _coef_in(dev, F):
    c = torch.zeros((2, F), dtype=torch.float64, device=dev)
    c[0, 4], c[1, 1], c[1, 5] = -1.1107592869834308, -0.14540553723951796, -1.0234639833519243
    return c


@pytest.mark.parametrize("N,T,Nr,Tr,gblocks", [
    (100_000, 200, 100_000, 200, 0),
    (100_000, 200, 100_000, 200, 196),
    (100_000, 200, 100_000, 200, 1),
    (3_001, 60, 5_003, 37, 0),
    (64, 20, 65, 33, 7),
    (20_000, 113, 1_000, 500, 300),
])
def test_fused_matches_separate_calls(dev, N, T, Nr, Tr, gblocks):
    from insite_amd import ops
    disc, rc, bits = _cohorts(dev, N, T, Nr, Tr)
    if N <= 5_000:   # ragged rows (incl. < 5: no contribution) on the small cohorts
        g = torch.Generator(device=dev)
        g.manual_seed(N)
        disc.rows = torch.randint(0, T - 1, (N,), generator=g, device=dev, dtype=torch.int32)
    lib = disc.lib
    cin = _coef_in(dev, lib.n_terms)
    (coef, mask, iters, G, b), y = ops.fit_rollout(disc.x, disc.u, disc.arm, disc.rows, disc.dt, lib, 0.1, 0.5,
                                                   rc.y0, rc.u, bits, cin, rc.dt, method="rk4",
                                                   gram_blocks=gblocks)
    c2, m2, _, G2, b2 = ops.sindy_fit(disc.x, disc.u, disc.arm, disc.rows, disc.dt, lib, 0.1, 0.5, layout="time")
    y2 = ops.rollout(rc.y0, rc.u, bits, cin, lib, rc.dt, method="rk4", T=Tr, layout="time_bits")
    torch.cuda.synchronize()
    assert torch.equal(y, y2), "fused rollout differs from insite_rollout_f64"
    np.testing.assert_allclose(G.cpu().numpy(), G2.cpu().numpy(), rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(b.cpu().numpy(), b2.cpu().numpy(), rtol=1e-12, atol=1e-9)
    assert torch.equal(mask, m2)
    assert (coef - c2).abs().max().item() < 1e-10
    # the discovery half against the oracle (small cohorts: the oracle's vectorised Gram finishes in seconds)
    if N <= 20_000:
        x = disc.x[:, :N].t().contiguous().cpu().numpy()
        rows = disc.rows.cpu().numpy()
        exps = lib.exps.astype(np.int64)
        u, arm = disc.u.cpu().numpy(), disc.arm.cpu().numpy().astype(np.int64)
        if N <= 5_000:
            Gr, br = R.gram_moments(x, u, arm, rows, disc.dt, exps)
        else:
            assert (rows == T - 2).all()
            Gr, br = R.gram_moments_vectorized(x, u, arm, T - 2, disc.dt, exps)
        np.testing.assert_allclose(G.cpu().numpy(), Gr, rtol=1e-10, atol=1e-8)
        cr = np.stack([R.stlsq_gram(Gr[a], br[a], 0.1, 0.5)[0] for a in range(2)])
        assert np.array_equal(mask.cpu().numpy() != 0, cr != 0)
        assert np.max(np.abs(coef.cpu().numpy() - cr)) < 1e-8


def test_fused_rollout_against_oracle_sample(dev):
    """The rollout half against the oracle's stage-by-stage RK4 (sampled rows, rtol 1e-11)."""
    from insite_amd import ops
    disc, rc, bits = _cohorts(dev, 2_000, 60, 9_000, 200, seed=11)
    lib = disc.lib
    cin = _coef_in(dev, lib.n_terms)
    _, y = ops.fit_rollout(disc.x, disc.u, disc.arm, disc.rows, disc.dt, lib, 0.1, 0.5, rc.y0, rc.u, bits, cin,
                           rc.dt, method="rk4")
    torch.cuda.synchronize()
    idx = np.unique(np.concatenate([np.arange(0, 9_000, 37), np.arange(8_960, 9_000)]))
    it = torch.as_tensor(idx, device=dev)
    arm8 = torch.stack([(bits[:, i // 32] >> (i % 32)) & 1 for i in idx.tolist()], 1).to(torch.int64)
    ref = R.rollout(rc.y0[it].cpu().numpy(), rc.u[it].cpu().numpy(), arm8.t().contiguous().cpu().numpy()[:, :200],
                    cin.cpu().numpy(), lib.exps.astype(np.int64), rc.dt, method="rk4")
    got = y.index_select(1, it).t().cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-11)


def test_fused_is_bitwise_reproducible_and_gram_only(dev):
    from insite_amd import ops
    disc, rc, bits = _cohorts(dev, 30_000, 200, 30_000, 200, seed=21)
    lib = disc.lib
    cin = _coef_in(dev, lib.n_terms)
    outs = [ops.fit_rollout(disc.x, disc.u, disc.arm, disc.rows, disc.dt, lib, 0.1, 0.5, rc.y0, rc.u, bits, cin,
                            rc.dt, method="euler5", gram_blocks=150) for _ in range(2)]
    torch.cuda.synchronize()
    (a, ya), (b_, yb) = outs
    assert torch.equal(ya, yb) and all(torch.equal(p, q) for p, q in zip(a, b_))
    # gram only: an empty rollout cohort (n_rows = 0)
    empty = torch.empty(0, dtype=torch.float64, device=dev)
    (coef, mask, _, G, _), _ = ops.fit_rollout(disc.x, disc.u, disc.arm, disc.rows, disc.dt, lib, 0.1, 0.5, empty,
                                               torch.empty((0, 2), dtype=torch.float64, device=dev),
                                               torch.zeros((200, 1), dtype=torch.int32, device=dev), cin, rc.dt,
                                               method="rk4", gram_blocks=150)
    torch.cuda.synchronize()
    assert torch.equal(G, a[3]) and torch.equal(coef, a[0]) and torch.equal(mask, a[1])


def test_fused_refuses_unsupported_shapes(dev):
    from insite_amd import ops, _lib
    from insite_amd.library import polynomial_library
    disc, rc, bits = _cohorts(dev, 1_000, 60, 1_000, 60)
    lib1 = polynomial_library(1, 2, True)   # 4 terms: the fused STLSQ is F = 7 only
    u1 = disc.u[:, :1].contiguous()
    with pytest.raises(_lib.InsiteError):
        ops.fit_rollout(disc.x, u1, disc.arm, disc.rows, disc.dt, lib1, 0.1, 0.5, rc.y0, rc.u[:, :1].contiguous(),
                        bits, torch.zeros((2, lib1.n_terms), dtype=torch.float64, device=dev), rc.dt)


@pytest.mark.parametrize("N,T,Nr,Tr,gblocks", [
    (100_000, 200, 100_000, 200, 0),
    (3_001, 60, 5_003, 37, 0),
    (64, 20, 65, 33, 7),
])
def test_deferred_stream_matches_separate_calls(dev, N, T, Nr, Tr, gblocks):
    """insite_fit_rollout_deferred_f64 over a stream of three cohorts plus the flush call: call k streams cohort
    k's Gram into slot k % 2 and finalises cohort k - 1 (coef / mask / iters / G / b equal to insite_sindy_fit_f64
    -- G|b bitwise those of insite_fit_rollout_f64 with the same gram_blocks, whose tail sums the same partials in
    the same order); every call's y bitwise insite_rollout_f64's.  The oracle checks the small cohorts' fits."""
    from insite_amd import cohort, ops
    lib = None
    discs = []
    for k in range(3):
        d = cohort.synthetic_pkpd(N, T, seed=11 + k, device=dev, equation="EQ_4_C", layout="time")
        if N <= 5_000:
            g = torch.Generator(device=dev)
            g.manual_seed(N + k)
            d.rows = torch.randint(0, T - 1, (N,), generator=g, device=dev, dtype=torch.int32)
        discs.append(d)
        lib = d.lib
    _, rc, bits = _cohorts(dev, 64, T, Nr, Tr, seed=21)
    F = lib.n_terms
    cin = _coef_in(dev, F)
    ws = ops.Workspace()
    f64 = torch.float64
    outs = [(torch.zeros((2, F), dtype=f64, device=dev), torch.zeros((2, F), dtype=torch.int8, device=dev),
             torch.zeros((2,), dtype=torch.int32, device=dev), torch.zeros((2, F, F), dtype=f64, device=dev),
             torch.zeros((2, F), dtype=f64, device=dev)) for _ in range(3)]
    y_ref = ops.rollout(rc.y0, rc.u, bits, cin, lib, rc.dt, method="rk4", T=Tr, layout="time_bits")
    for k in range(4):   # k = 3: the flush (no cohort streamed, no rollout), finalising cohort 2
        d = discs[min(k, 2)]
        n = N if k < 3 else 0
        (_, _, _, _, _), y = ops.fit_rollout_deferred(
            d.x[:, :n] if n else d.x[:, :0], d.u[:n], d.arm[:n], d.rows[:n], d.dt, lib, 0.1, 0.5,
            rc.y0 if k < 3 else rc.y0[:0], rc.u if k < 3 else rc.u[:0], bits, cin, rc.dt, k % 2, k > 0, ws,
            method="rk4", T=Tr, out=outs[k - 1] if k > 0 else outs[2], gram_blocks=gblocks)
        if k < 3:
            torch.cuda.synchronize()
            assert torch.equal(y, y_ref), f"call {k}: deferred rollout differs from insite_rollout_f64"
    torch.cuda.synchronize()
    for k in range(3):
        d = discs[k]
        coef, mask, iters, G, b = outs[k]
        (c1, m1, _, G1, b1), _ = ops.fit_rollout(d.x, d.u, d.arm, d.rows, d.dt, lib, 0.1, 0.5, rc.y0, rc.u, bits,
                                                 cin, rc.dt, method="rk4", gram_blocks=gblocks, T=Tr)
        c2, m2, _, G2, b2 = ops.sindy_fit(d.x, d.u, d.arm, d.rows, d.dt, lib, 0.1, 0.5, layout="time")
        torch.cuda.synchronize()
        assert torch.equal(G, G1) and torch.equal(b, b1), f"cohort {k}: deferred G|b differ from the in-launch tail"
        assert torch.equal(coef, c1) and torch.equal(mask, m1)
        np.testing.assert_allclose(G.cpu().numpy(), G2.cpu().numpy(), rtol=1e-12, atol=1e-9)
        assert torch.equal(mask, m2)
        assert (coef - c2).abs().max().item() < 1e-10
        if N <= 5_000:
            x = d.x[:, :N].t().contiguous().cpu().numpy()
            Gr, br = R.gram_moments(x, d.u.cpu().numpy(), d.arm.cpu().numpy().astype(np.int64),
                                    d.rows.cpu().numpy(), d.dt, lib.exps.astype(np.int64))
            np.testing.assert_allclose(G.cpu().numpy(), Gr, rtol=1e-10, atol=1e-8)
            cr = np.stack([R.stlsq_gram(Gr[a], br[a], 0.1, 0.5)[0] for a in range(2)])
            assert np.array_equal(mask.cpu().numpy() != 0, cr != 0)
            assert np.max(np.abs(coef.cpu().numpy() - cr)) < 1e-8
