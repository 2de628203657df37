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


# ---------------------------------------------------------------------------------- ablation models
def _joint_cohort(n=80, seed=1):
    """EQ_4_C in multilabel mode, the joint ("one ODE") model fitted on it (sindy.py:203; pkpd/utils.py:486-497)."""
    coll = R.make_collection("EQ_4_C", {"train": n, "val": 4, "test": 4}, seed=seed, with_tests=False,
                             treatment_mode="multilabel")
    tr = coll["train"]
    x, inputs, stat, rows = R.de_format_joint(tr.data, tr.scaling_params)
    ex = R.poly_library(1 + inputs.shape[-1] + stat.shape[1], 2, True)
    Z, Y = R.build_regression_joint(x, inputs, stat, rows, DT)
    c, _, _ = R.stlsq(R.eval_library(ex, Z), Y, 0.1, 0.5)
    prev, _ = R.unscale_inputs(tr.data, tr.scaling_params)
    code = inputs[..., 0].astype(np.int64)
    return prev, code, stat, c[None, :], ex


def test_joint_fold_equals_literal_rhs():
    """The joint model's per-combination fold (coef_terms) is the literal RHS on [treatment_k, statics]
    (R.rollout_inputs, sindy.py:317-322), Euler-5."""
    prev, code, stat, c0, ex = _joint_cohort()
    c = c0.copy()
    for p in range(5):
        got = Q.euler5_rollout(prev[p, 0], code[p], stat[p], c, ex, DT, code.shape[1], n_inputs=1)
        ref = R.rollout_inputs(prev[p:p + 1, 0], stat[p:p + 1], code[p:p + 1, :, None].astype(np.float64), c[0], ex,
                               DT)[0]
        np.testing.assert_allclose(got, ref, rtol=1e-12)


@pytest.mark.parametrize("kind", ["joint", "degree4"])
def test_ablation_gradient_matches_finite_differences(cohort, kind):
    if kind == "joint":
        prev, code, stat, c0, ex = _joint_cohort()
        V, arms, u, n_in = prev[3], code[3], stat[3], 1
    else:
        x, u_, arm, _ = cohort
        ex = R.poly_library(3, 4, False)
        rng = np.random.default_rng(0)
        c0 = np.zeros((2, ex.shape[0]))
        c0[0, 4] = -1.0                                   # x0 u0 ... plus small higher-degree terms
        for j in np.nonzero(ex[:, 0] >= 2)[0][:4]:
            c0[:, j] = rng.normal(0, 0.05, 2)
        c0[1, 1] = -0.15
        # a unit-scale series so the x^2..x^4 terms stay O(1) over the window
        V, arms, u, n_in = x[3] / x[3].max(), np.where(np.arange(x.shape[1]) < 30, arm[3], 1 - arm[3]), u_[3], 0
    pb = Q.PatientProblem(V, arms, u, c0, ex, 45, DT, 10.0, n_inputs=n_in)
    assert pb.D == (4 if kind == "degree4" else 1) and len(pb.terms) >= 2
    pb.norm = 0.7
    c = pb.c0 * np.linspace(0.95, 1.05, pb.c0.size)
    f, g = pb.value_and_grad(c)
    eye = np.eye(c.size)
    step = 1e-6 * np.maximum(np.abs(c), 1e-3)
    fd = np.array([(pb.value_and_grad(c + step[i] * eye[i])[0] - pb.value_and_grad(c - step[i] * eye[i])[0])
                   / (2 * step[i]) for i in range(c.size)])
    assert np.abs(g - fd).max() <= 1e-5 * np.abs(g).max()


def test_joint_refinement_reaches_scipys_optimum():
    prev, code, stat, c0, ex = _joint_cohort()
    p, sl, tau = 2, 59, 5
    preds, c, status, it = Q.refine_patient(prev[p], code[p], stat[p], sl, c0, ex, DT, 10.0, tau, n_inputs=1)
    assert status in (0, 2, 3) and it > 0
    pb = Q.PatientProblem(prev[p], code[p], stat[p], c0, ex, sl - tau, DT, 10.0, n_inputs=1)
    pb.norm = 2.5 * pb.value_and_grad(pb.c0)[0]
    r = minimize(pb.value_and_grad, pb.c0.copy(), jac=True, method="BFGS", options={"gtol": 1e-8})
    mine = np.array([c.flat[t[0]] for t in pb.terms])
    assert pb.value_and_grad(mine)[0] <= r.fun * (1 + 1e-6) + 1e-12
