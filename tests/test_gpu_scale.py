"""GPU vs oracle at the BASELINE configuration sizes (VERDICT r1 "oracle parity at config size").

* C2 discovery: insite_sindy_fit_f64 on the bench's own 100k x 200 EQ_4_C cohort (cohort.synthetic_pkpd,
  both HBM layouts) against the oracle's vectorised Gram + Gram-form STLSQ (oracle/insite_ref.py):
  Gram to rtol 1e-10, identical support, coefficient L-inf < 1e-8 (north star).
* North-star rollout: the 1M x 500 bit-arm RK4 rollout, checked against the oracle's stage-by-stage
  RK4 on a sampled subset of 4096 patients spread over the whole launch (every 64-patient tile family,
  the last partial bit word): rtol 1e-11, trajectory RMSE <= 1e-6.
"""
import numpy as np
import pytest
import torch

from oracle import insite_ref as R

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("layout", ["time", "patient"])
def test_c2_discovery_matches_oracle_at_config_size(dev, layout):
    from insite_amd import cohort, ops
    N, T = 100_000, 200
    coh = cohort.synthetic_pkpd(N, T, seed=1000, device=dev, equation="EQ_4_C", layout=layout)
    coef, mask, _, G, b = ops.sindy_fit(coh.x, coh.u, coh.arm, coh.rows, coh.dt, coh.lib, 0.1, 0.5, layout=layout)
    x = (coh.x[:, :N].t() if layout == "time" else coh.x[:, :T]).contiguous().cpu().numpy()
    u, arm = coh.u.cpu().numpy(), coh.arm.cpu().numpy().astype(np.int64)
    exps = coh.lib.exps.astype(np.int64)
    Gr, br = R.gram_moments_vectorized(x, u, arm, T - 2, coh.dt, exps)
    np.testing.assert_allclose(G.cpu().numpy(), Gr, rtol=1e-10, atol=1e-6)
    np.testing.assert_allclose(b.cpu().numpy(), br, rtol=1e-10, atol=1e-6)
    cr = np.stack([R.stlsq_gram(Gr[a], br[a], 0.1, 0.5)[0] for a in range(2)])
    assert np.array_equal(mask.cpu().numpy() != 0, cr != 0)
    assert np.max(np.abs(coef.cpu().numpy() - cr)) < 1e-8
    assert [list(np.nonzero(c)[0]) for c in cr] == [[4], [1, 5]]      # the EQ_4_C support


def test_north_star_rollout_sampled_against_oracle(dev):
    from insite_amd import ops
    from insite_amd.library import polynomial_library
    Nn, Tn = 1_000_000, 500
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    y0 = torch.rand(Nn, generator=g, device=dev, dtype=torch.float64) * 49 + 1
    u = torch.rand((Nn, 2), generator=g, device=dev, dtype=torch.float64) * 0.1 + 0.45
    flip = torch.randint(0, Tn, (Nn,), generator=g, device=dev)
    arm8 = (torch.arange(Tn, device=dev)[:, None] >= flip[None, :]).to(torch.int8)
    bits = ops.pack_arm_bits(arm8, Nn)
    lib = polynomial_library(2, 2, True)
    coef = torch.zeros((2, lib.n_terms), dtype=torch.float64, device=dev)
    coef[0, 4], coef[1, 1], coef[1, 5] = -1.1107592869834308, -0.14540553723951796, -1.0234639833519243
    y = ops.rollout(y0, u, bits, coef, lib, 10.0 / Tn, method="rk4", layout="time_bits")
    torch.cuda.synchronize()
    rng = np.random.default_rng(3)
    idx = np.unique(np.concatenate([rng.choice(Nn, 4000, replace=False), np.arange(64), np.arange(Nn - 96, Nn)]))
    it = torch.as_tensor(idx, device=dev)
    arms = arm8.index_select(1, it).t().contiguous().cpu().numpy()
    ref = R.rollout(y0[it].cpu().numpy(), u[it].cpu().numpy(), arms, coef.cpu().numpy(),
                    lib.exps.astype(np.int64), 10.0 / Tn, method="rk4")
    got = y.index_select(1, it).t().cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-11)
    assert np.sqrt(np.mean((got - ref) ** 2)) <= 1e-6
