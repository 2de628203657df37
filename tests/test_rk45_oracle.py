"""CPU tests: the RK45 restatement (oracle/rk45_ref.py, configuration C5) is pinned against scipy's
solve_ivp(method='RK45') — the third-party algorithm it restates (scipy 1.15.3, importable here)."""
import numpy as np
import pytest
from scipy.integrate import solve_ivp

from oracle import insite_ref as R
from oracle import rk45_ref as K


@pytest.mark.parametrize("seed", range(4))
def test_rk45_interval_matches_solve_ivp(seed):
    rng = np.random.default_rng(seed)
    for _ in range(50):
        al, be = rng.normal(0, 2), rng.normal(-1.0, 0.7)
        y0 = rng.uniform(-5, 50)
        t0 = rng.uniform(0, 5)
        t1 = t0 + rng.uniform(1e-4, 2.0)
        y, n = K.rk45_interval(lambda v: al + be * v, y0, t0, t1)
        s = solve_ivp(lambda t, v: al + be * v, (t0, t1), [y0], method="RK45", rtol=K.RTOL, atol=K.ATOL)
        assert abs(y - s.y[0, -1]) <= 1e-13 * max(1.0, abs(s.y[0, -1]))
        # the controller takes the same accepted steps (solve_ivp stores one column per accepted step)
        assert n >= s.t.size - 1


def test_rk45_tracks_the_exact_solution():
    al, be, y0 = 1.3, -0.8, 20.0
    y, _ = K.rk45_interval(lambda v: al + be * v, y0, 0.0, 3.0)
    exact = (y0 + al / be) * np.exp(be * 3.0) - al / be
    assert abs(y - exact) < 1e-7 * abs(exact)


def test_zero_length_interval_is_identity():
    y, n = K.rk45_interval(lambda v: -v, 3.0, 1.0, 1.0)
    assert y == 3.0 and n == 0


def test_irregular_grid_distribution():
    t, n = K.irregular_grid(500, np.random.default_rng(0))
    assert n.min() >= 20 and n.max() <= 60 and t.shape == (500, 60)
    for p in range(500):
        g = t[p, : n[p]]
        assert g[0] == 0.0 and np.all(np.diff(g) >= 0) and g[-1] <= 10.0
        assert np.isnan(t[p, n[p]:]).all()


def test_rollout_rk45_uses_per_interval_arms_and_drop_filter():
    ex = R.poly_library(3, 2, True)
    coef = np.zeros((2, 7))
    coef[0, 4] = -1.1
    coef[1, 1] = -0.15
    coef[1, 5] = -1.0
    coef[1, 6] = 5e-4                        # below the 1e-3 RHS filter (utils.py:388)
    u = np.array([[0.5, 0.6]])
    t = np.array([[0.0, 0.5, 1.7, 2.0]])
    arm = np.array([[0, 1, 0, 0]])
    y, steps = K.rollout_rk45(np.array([10.0]), u, arm, t, np.array([4]), coef, ex)
    rates = [-1.1 * 0.5, -0.15 - 1.0 * 0.6]
    ref = 10.0
    for k in range(3):
        ref = ref * np.exp(rates[arm[0, k]] * (t[0, k + 1] - t[0, k]))
        assert abs(y[0, k] - ref) < 1e-7 * ref
    assert steps[0] > 0
