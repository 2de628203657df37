"""CPU tests of the INSITE refinement restatement (oracle/insite_refine_ref.py; reference
sindy.py:433-715, 767-794).  jax is absent, so the BFGS restatement is pinned by (i) exact gradients
(finite differences), (ii) scipy.optimize.minimize(BFGS) reaching the same optimum of the same objective,
(iii) the reference's control flow (skip when seq_len <= tau, status-3 fallback)."""
import numpy as np
import pytest
from scipy.optimize import minimize

from oracle import insite_ref as R
from oracle import insite_refine_ref as Q

EX = R.poly_library(3, 2, True)
DT = R.STANDARD_DT


@pytest.fixture(scope="module")
def cohort():
    coll = R.make_collection("EQ_4_C", {"train": 120, "val": 4, "test": 4}, seed=1, with_tests=False)
    tr = coll["train"]
    x, u, arm, rows = R.de_format(tr.data, tr.scaling_params)
    G, b = R.gram_moments(x, u, arm, rows, DT, EX)
    c0 = np.stack([R.stlsq_gram(G[a], b[a], 0.1, 0.5)[0] for a in range(2)])
    return x, u, arm, c0


def test_gradient_matches_finite_differences(cohort):
    x, u, arm, c0 = cohort
    arms = np.full(x.shape[1], arm[3])
    arms[30:] = 1 - arm[3]                       # a switch inside the window
    pb = Q.PatientProblem(x[3], arms, u[3], c0, EX, 45, DT, 10.0)
    pb.norm = 0.7
    c = pb.c0 * np.array([1.03, 0.9, 1.1])
    f, g = pb.value_and_grad(c)
    eye = np.eye(c.size)
    fd = np.array([(pb.value_and_grad(c + 1e-6 * eye[i])[0] - pb.value_and_grad(c - 1e-6 * eye[i])[0]) / 2e-6
                   for i in range(c.size)])
    assert np.abs(g - fd).max() <= 1e-6 * np.abs(g).max()


@pytest.mark.parametrize("p", range(6))
def test_bfgs_reaches_scipys_optimum(cohort, p):
    x, u, arm, c0 = cohort
    arms = np.full(x.shape[1], arm[p])
    sl, tau = 59, 5
    preds, c, status, it = Q.refine_patient(x[p], arms, u[p], sl, c0, EX, DT, 10.0, tau)
    assert status == 0 and it > 0
    pb = Q.PatientProblem(x[p], arms, u[p], c0, EX, sl - tau, DT, 10.0)
    pb.norm = 2.5 * pb.value_and_grad(pb.c0)[0]
    r = minimize(pb.value_and_grad, pb.c0.copy(), jac=True, method="BFGS", options={"gtol": 1e-8})
    mine = np.array([c.flat[t[0]] for t in pb.terms])
    assert np.abs(mine - r.x).max() < 1e-5
    assert pb.value_and_grad(mine)[0] <= r.fun * (1 + 1e-9) + 1e-15
    # inactive coefficients never move; predictions are the refined model's Euler-5 scan
    assert np.array_equal(c[np.abs(c0) <= 1e-3], c0[np.abs(c0) <= 1e-3])
    assert np.allclose(preds, Q.euler5_rollout(x[p, 0], arms, u[p], c, EX, DT, x.shape[1]))


def test_short_rows_are_not_refined(cohort):
    x, u, arm, c0 = cohort
    arms = np.full(x.shape[1], arm[0])
    preds, c, status, it = Q.refine_patient(x[0], arms, u[0], 5, c0, EX, DT, 10.0, 5)
    assert status == -1 and it == 0 and np.array_equal(c, c0)
    assert np.allclose(preds, Q.euler5_rollout(x[0, 0], arms, u[0], c0, EX, DT, x.shape[1]))


def test_refinement_reduces_the_fit_error(cohort):
    """The point of INSITE: the individualised model fits the observed prefix better."""
    x, u, arm, c0 = cohort
    better = 0
    for p in range(10):
        arms = np.full(x.shape[1], arm[p])
        preds, c, status, _ = Q.refine_patient(x[p], arms, u[p], 59, c0, EX, DT, 10.0, 5)
        base = Q.euler5_rollout(x[p, 0], arms, u[p], c0, EX, DT, x.shape[1])
        K = 54
        e_ref = np.mean((x[p, 1:K + 1] - preds[:K]) ** 2)
        e_glob = np.mean((x[p, 1:K + 1] - base[:K]) ** 2)
        better += e_ref <= e_glob
    assert better == 10


def test_line_search_helpers():
    # quadratic/cubic interpolants recover the minimiser of an exact quadratic / cubic
    f = lambda t: (t - 0.3) ** 2
    assert abs(Q._quadmin(0.0, f(0.0), -0.6, 1.0, f(1.0)) - 0.3) < 1e-12
    g = lambda t: t ** 3 - 2 * t ** 2 + 0.5 * t
    xm = Q._cubicmin(0.0, g(0.0), 0.5, 2.0, g(2.0), 1.0, g(1.0))
    assert abs(xm - (4 + np.sqrt(16 - 6)) / 6) < 1e-12
