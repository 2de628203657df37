"""GPU parity of the treatment-segment discovery (the cancer_sim / EQ_5 path) through
the C ABI (insite_gram_segments_f64 / insite_sindy_fit_segments_f64) and the 4-arm rollout, against
oracle/segments_ref.py.

Tolerances (north star, BASELINE.json): Gram sums rtol 1e-10 (fp64, different association order);
identical support and coefficient L-inf < 1e-8; trajectory RMSE <= 1e-6.
"""
import numpy as np
import pytest
import torch

from oracle import insite_ref as R
from oracle import segments_ref as S

pytestmark = pytest.mark.gpu

COEF_TOL = 1e-8


def _t(a, dev, dtype=None):
    return torch.tensor(np.ascontiguousarray(a), device=dev, dtype=dtype)


def _lib(n_statics):
    from insite_amd.library import polynomial_library
    return polynomial_library(n_statics, 2, True)


def _poisoned(x, arm, sl, n_arms):
    """What the reference never reads is poisoned: samples past seq_len are NaN, arms from seq_len
    on are changed (a stray read would break the sums or the segment cuts)."""
    xp, ap = x.copy(), arm.copy()
    for i in range(x.shape[0]):
        xp[i, sl[i] + 1:] = np.nan
        ap[i, sl[i]:] = (ap[i, sl[i]:] + 1) % n_arms
    return xp, ap


def _layout(x, arm, layout, dev, pad=3):
    if layout == "patient":
        return _t(x, dev), _t(arm, dev, torch.int8)
    N = x.shape[0]
    xt = np.full((x.shape[1], N + pad), np.nan)
    xt[:, :N] = x.T
    at = np.zeros((arm.shape[1], N + pad), dtype=np.int8)
    at[:, :N] = arm.T
    return _t(xt, dev), _t(at, dev, torch.int8)


def _close(got, ref, rtol=1e-10):
    np.testing.assert_allclose(got, ref, rtol=rtol, atol=rtol * max(1.0, float(np.abs(ref).max())))


@pytest.mark.parametrize("layout", ["patient", "time"])
@pytest.mark.parametrize("fd", ["order1", "smoothed1"])
@pytest.mark.parametrize("n_statics,n_arms", [(1, 4), (2, 4), (2, 3), (1, 2), (1, 1)])
def test_gram_segments_matches_oracle(dev, layout, fd, n_statics, n_arms):
    from insite_amd import ops
    rng = np.random.default_rng(11 + n_arms)
    N, T = 613, 40
    coef = S.TRUE_COEF_U1[:n_arms] if n_statics == 1 else rng.normal(0, 0.1, size=(n_arms, 7))
    x, u, arm, sl = S.synthetic_cohort(N, T, rng, switch_p=0.2, noise=0.01, coef=coef, n_statics=n_statics, min_len=0)
    sl[:6] = [0, 1, 2, 3, T, T - 1]
    arm[4, -1] = (arm[4, -2] + 1) % n_arms if n_arms > 1 else 0     # a switch at the last step
    lib = _lib(n_statics)
    G_ref, b_ref, cnt = S.gram_segments(x, u, arm, sl, 0.1, lib.exps.astype(np.int64), n_arms=n_arms, fd=fd)
    xp, ap = _poisoned(x, arm, sl, n_arms)
    xd, ad = _layout(xp, ap, layout, dev)
    G, b = ops.gram_segments(xd, ad, _t(sl, dev, torch.int32), _t(u, dev), 0.1, lib, n_arms=n_arms, fd=fd,
                             layout=layout)
    torch.cuda.synchronize()
    _close(G.cpu().numpy(), G_ref)
    _close(b.cpu().numpy(), b_ref)
    np.testing.assert_array_equal(G.cpu().numpy()[:, 0, 0], cnt)


@pytest.mark.parametrize("fd", ["order1", "smoothed1"])
@pytest.mark.parametrize("n_statics", [1, 2])
def test_sindy_fit_segments_matches_oracle(dev, fd, n_statics):
    """Support, coefficients and iteration counts of the four per-arm STLSQ fits at the reference's
    cancer_sim / EQ_5 threshold 0.001 (config/config.yaml:20-22)."""
    from insite_amd import ops
    rng = np.random.default_rng(5 + n_statics)
    coef = S.TRUE_COEF_U1 if n_statics == 1 else rng.normal(0, 0.1, size=(4, 7))
    x, u, arm, sl = S.synthetic_cohort(900, 60, rng, switch_p=0.1, noise=0.005, dt=0.05, coef=coef,
                                       n_statics=n_statics, min_len=10)
    c_ref, ind_ref, it_ref, _ = S.sindy_fit_segments(x, u, arm, sl, 0.05, threshold=1e-3, alpha=0.5, fd=fd)
    coef_d, mask, iters, G, b = ops.sindy_fit_segments(_t(x, dev), _t(arm, dev, torch.int8), _t(sl, dev, torch.int32),
                                                       _t(u, dev), 0.05, _lib(n_statics), 1e-3, 0.5, fd=fd)
    torch.cuda.synchronize()
    assert np.array_equal(mask.cpu().numpy().astype(bool), ind_ref)
    assert np.max(np.abs(coef_d.cpu().numpy() - c_ref)) < COEF_TOL
    np.testing.assert_array_equal(iters.cpu().numpy(), it_ref)


def test_planted_system_recovered_time_major(dev):
    from insite_amd import ops
    rng = np.random.default_rng(3)
    x, u, arm, sl = S.synthetic_cohort(600, 200, rng, switch_p=0.05, dt=0.01)
    xd, ad = _layout(x, arm, "time", dev)
    coef, mask, iters, _, _ = ops.sindy_fit_segments(xd, ad, _t(sl, dev, torch.int32), _t(u, dev), 0.01, _lib(1), 0.1,
                                                     0.5, layout="time")
    np.testing.assert_array_equal(mask.cpu().numpy().astype(bool), S.TRUE_COEF_U1 != 0)
    assert np.max(np.abs(coef.cpu().numpy() - S.TRUE_COEF_U1)) < 0.02


def test_single_arm_cohort_leaves_other_arms_empty(dev):
    from insite_amd import ops
    rng = np.random.default_rng(8)
    x, u, arm, sl = S.synthetic_cohort(100, 20, rng, switch_p=0.0)
    arm[:] = 2
    G, b = ops.gram_segments(_t(x, dev), _t(arm, dev, torch.int8), _t(sl, dev, torch.int32), _t(u, dev), 0.1, _lib(1))
    G = G.cpu().numpy()
    assert np.all(G[[0, 1, 3]] == 0) and G[2, 0, 0] == 100 * 21
    G_ref, b_ref, _ = S.gram_segments(x, u, arm, sl, 0.1, _lib(1).exps.astype(np.int64))
    _close(G, G_ref)


def test_large_cohort_properties_time_major(dev):
    """1M patients x 60 steps generated on the device: per-arm sample counts equal the closed form
    (own samples + one closing sample per segment), G is symmetric, runs are bitwise repeatable."""
    from insite_amd import ops
    N, T = 1_000_000, 60
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    x = torch.rand((T + 1, N), generator=g, device=dev, dtype=torch.float64) + 1.0
    arm = torch.randint(0, 4, (T, N), generator=g, device=dev, dtype=torch.int8)
    sl = torch.randint(0, T + 1, (N,), generator=g, device=dev, dtype=torch.int32)
    u = torch.rand((N, 2), generator=g, device=dev, dtype=torch.float64)
    lib = _lib(2)
    G1, b1 = ops.gram_segments(x, arm, sl, u, 0.1, lib, layout="time")
    G2, b2 = ops.gram_segments(x, arm, sl, u, 0.1, lib, layout="time")
    assert torch.equal(G1, G2) and torch.equal(b1, b2)
    k = torch.arange(T + 1, device=dev)[:, None]
    L = sl.to(torch.int64)[None, :]
    a = torch.full((T + 1, N), -1, dtype=torch.int64, device=dev)
    a[:T] = torch.where(k[:T] < L, arm.to(torch.int64), -1)
    prev = torch.full_like(a, -1)
    prev[1:] = a[:T]
    close = (prev >= 0) & (a != prev)
    for q in range(4):
        cnt = int((a == q).sum().item()) + int((close & (prev == q)).sum().item())
        assert G1[q, 0, 0].item() == cnt
    assert torch.equal(G1, G1.transpose(1, 2))
    assert bool(torch.isfinite(G1).all()) and bool(torch.isfinite(b1).all())


def test_four_arm_rollout_matches_oracle(dev):
    """lax.switch(argmax(treatment)) over four arms (sindy.py:307-312) with per-step arms: the rollout
    kernel at NARM = 4 against the oracle's Euler-5 and RK4."""
    from insite_amd import ops
    rng = np.random.default_rng(9)
    x, u, arm, sl = S.synthetic_cohort(333, 50, rng, switch_p=0.2, dt=0.1)
    lib = _lib(1)
    exps = lib.exps.astype(np.int64)
    for method in ("euler5", "rk4"):
        y_ref = R.rollout(x[:, 0], u, arm, S.TRUE_COEF_U1, exps, 0.1, method=method)
        y = ops.rollout(_t(x[:, 0], dev), _t(u, dev), _t(arm, dev, torch.int8), _t(S.TRUE_COEF_U1, dev), lib, 0.1,
                        method=method)
        torch.cuda.synchronize()
        yh = y.cpu().numpy()
        assert np.sqrt(np.mean((yh - y_ref) ** 2)) <= 1e-6
        np.testing.assert_allclose(yh, y_ref, rtol=1e-11)


class _Subset:
    """A processed dataset with the reference layout (pkpd/dataset.py / continuous/dataset.py): identity
    scaling so the unscaled arrays are the synthetic cohort itself; 4-arm one-hot treatments."""

    def __init__(self, x, u, arm, sl):
        N, T1 = x.shape
        T = T1 - 1
        self.subset_name = "train"
        self.norm_const = 50.0
        self.scaling_params = {"output_means": 0.0, "output_stds": 1.0, "input_means": np.zeros(1 + u.shape[1]),
                               "inputs_stds": np.ones(1 + u.shape[1])}
        self.data = {"prev_outputs": x[:, :T, None], "unscaled_outputs": x[:, 1:, None], "outputs": x[:, 1:, None],
                     "static_features": u, "current_treatments": np.eye(4)[arm],
                     "sequence_lengths": sl.astype(np.float64),
                     "active_entries": (np.arange(T)[None, :, None] < sl[:, None, None]).astype(np.float64)}


@pytest.mark.parametrize("name,n_statics", [("cancer_sim", 1), ("EQ_5_B", 2)])
def test_plugin_fit_and_predict_segments(dev, name, n_statics):
    """SINDY on a 4-arm dataset (sindy.py:160-216, 289-336): coefficients, support and the four-part
    equation string against the row-form oracle; predictions against the oracle rollout."""
    from insite_amd.sindy import SINDY
    rng = np.random.default_rng(21)
    coef = S.TRUE_COEF_U1 if n_statics == 1 else rng.normal(0, 0.1, size=(4, 7))
    x, u, arm, sl = S.synthetic_cohort(500, 60, rng, switch_p=0.1, noise=0.01, dt=1 / 6, coef=coef,
                                       n_statics=n_statics, min_len=20)
    args = {"model": {"dataset_name": name, "dim_treatments": 4, "dim_static_features": n_statics,
                      "dim_outcomes": 1, "sindy_threshold": 0.001, "sindy_alpha": 0.5},
            "dataset": {"projection_horizon": 5}, "exp": {"unscale_rmse": True, "percentage_rmse": True}}
    m = SINDY(args, device=dev)
    ds = _Subset(x, u, arm, sl)
    m.fit(ds)
    c_ref, ind_ref, _, exps = S.sindy_fit_segments(x, u, arm, sl, 1 / 6, threshold=1e-3, alpha=0.5)
    assert np.array_equal(m.joint_coefs != 0, ind_ref)
    assert np.max(np.abs(m.joint_coefs - c_ref)) < COEF_TOL
    assert m.global_equation_string.count("Treatment ") == 4
    p = m.get_predictions(ds)[..., 0]
    y_ref = R.rollout(x[:, 0], u, arm, np.where(np.abs(c_ref) > 1e-3, c_ref, 0.0), exps, 1 / 6)
    assert np.sqrt(np.mean((p - y_ref) ** 2)) <= 1e-6
