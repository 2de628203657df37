"""CPU restatement for the multi-state configuration C3 (TEST INFRASTRUCTURE ONLY — never imported by
the product package; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it).

C3 (BASELINE.json configs[2]) is build-defined: the reference repo has no multi-state
system.  It extends the reference's discovery semantics (pysindy SmoothedFiniteDifference + PolynomialLibrary
+ STLSQ, reference libs_m/ct/src/models/sindy.py:186-213) from one state to S states and its rollout
(odeint / RK4, pkpd/utils.py:68-94) to an S-dimensional state:

  * states x_1..x_5 (a 4-compartment PK chain feeding a tumour with a bilinear kill term) and one binary
    per-step treatment input a_k (Markov: a_0 ~ Bernoulli(0.3), switch with probability 0.01 per step);
  * library = pysindy PolynomialLibrary(degree=2, interaction_only=True) over the inputs (x_1..x_5, a):
    F = 22 columns in pysindy order (``insite_ref.poly_library(6)``); joint (not arm-split) regression with
    the treatment as an input column, as the reference's joint mode does (pkpd/utils.py:488-497);
  * derivative: savgol(5,3)-smoothed 4th-order FD per state over the patient's rows; the library sees the
    RAW states (the smoothing feeds x_dot only — pinned on the reference's one-state cohorts, see
    insite_ref.smoothed_fd4);
  * one STLSQ per target state on the shared Gram (insite_ref.stlsq_gram; pysindy fits targets separately);
  * rollout: RK4 (or Euler) of the discovered S-state system, treatment a_k held over interval k, RHS terms
    with |c| > 1e-3 (pkpd/utils.py:388), output = state after each interval (insite_ref.rollout convention).

Parity for C3 is against this restatement only ("parity unpinned" with respect to the reference: no
reference counterpart exists); the truth model is recovered exactly by it (tests/test_multistate_oracle.py).
"""
from __future__ import annotations

import numpy as np

from . import insite_ref as R

S_C3 = 5
INPUT_NAMES_C3 = ["x1", "x2", "x3", "x4", "x5", "a"]
RATES_C3 = {"k1": 1.2, "k2": 0.8, "k3": 0.5, "k4": 0.6, "k5": 0.1, "e": 0.4, "D": 2.0}
THRESHOLD_C3 = 0.05
ALPHA_C3 = 0.5
DT_C3 = 0.02


def c3_library():
    """Exponent table [22, 6] over (x1..x5, a) in pysindy order."""
    return R.poly_library(S_C3 + 1, 2, True)


def _col(exps, *idx):
    e = np.zeros(exps.shape[1], dtype=np.int64)
    for i in idx:
        e[i] += 1
    hit = np.nonzero((exps == e).all(axis=1))[0]
    return int(hit[0])


def c3_truth_coef(exps=None, rates=RATES_C3):
    """True coefficients [S, F] of the C3 system in the library basis:
        x1' = -k1 x1 + D a            x2' = k1 x1 - k2 x2          x3' = k2 x2 - k3 x3
        x4' =  k3 x3 - k4 x4          x5' = -k5 x5 - e x4 x5"""
    exps = c3_library() if exps is None else exps
    k = rates
    C = np.zeros((S_C3, exps.shape[0]))
    C[0, _col(exps, 0)] = -k["k1"]
    C[0, _col(exps, 5)] = k["D"]
    C[1, _col(exps, 0)] = k["k1"]
    C[1, _col(exps, 1)] = -k["k2"]
    C[2, _col(exps, 1)] = k["k2"]
    C[2, _col(exps, 2)] = -k["k3"]
    C[3, _col(exps, 2)] = k["k3"]
    C[3, _col(exps, 3)] = -k["k4"]
    C[4, _col(exps, 4)] = -k["k5"]
    C[4, _col(exps, 3, 4)] = -k["e"]
    return C


def eval_rhs(y, a, coef, exps, drop=R.RHS_COEF_EPS):
    """f(y, a)[N, S] = sum_j c[s, j] Theta_j(y, a) over |c| > drop.  y [N, S], a [N]."""
    Z = np.concatenate([y, np.asarray(a, dtype=np.float64)[:, None]], axis=1)
    th = R.eval_library(exps, Z)
    c = np.where(np.abs(coef) > drop, coef, 0.0)
    return th @ c.T


def treatment_markov(N, T, rng, p1=0.3, p_switch=0.01):
    a = np.empty((N, T), dtype=np.int8)
    cur = (rng.random(N) < p1).astype(np.int8)
    for k in range(T):
        a[:, k] = cur
        sw = rng.random(N) < p_switch
        cur = np.where(sw, 1 - cur, cur).astype(np.int8)
    return a


def c3_cohort(N, T, seed=2, dt=DT_C3, substeps=10, p1=0.3, p_switch=0.01):
    """Synthetic C3 cohort: x [N, T, S] (float32 storage, values rounded), treatments a [N, T] int8.
    Truth: the C3 system integrated with ``substeps`` RK4 steps per interval (fp64), x[:, 0] drawn
    x1..x4 ~ U(0, 1), x5 ~ U(1, 5)."""
    rng = np.random.default_rng(seed)
    exps = c3_library()
    C = c3_truth_coef(exps)
    y = np.stack([rng.uniform(0, 1, N), rng.uniform(0, 1, N), rng.uniform(0, 1, N), rng.uniform(0, 1, N),
                  rng.uniform(1, 5, N)], axis=1)
    a = treatment_markov(N, T, rng, p1, p_switch)
    x = np.empty((N, T, S_C3))
    h = dt / substeps
    for k in range(T):
        x[:, k] = y
        ak = a[:, k].astype(np.float64)
        for _ in range(substeps):
            k1 = eval_rhs(y, ak, C, exps, 0.0)
            k2 = eval_rhs(y + 0.5 * h * k1, ak, C, exps, 0.0)
            k3 = eval_rhs(y + 0.5 * h * k2, ak, C, exps, 0.0)
            k4 = eval_rhs(y + h * k3, ak, C, exps, 0.0)
            y = y + (h / 6.0) * (k1 + 2.0 * k2 + 2.0 * k3 + k4)
    return x.astype(np.float32), a


def ms_regression(x, a, L, dt):
    """Rows of one patient: library inputs Z [L, S+1] = (raw states, a) and targets xdot [L, S]
    (savgol(5,3) + FD4 per state, insite_ref.smoothed_fd4)."""
    X = np.asarray(x[:L], dtype=np.float64)
    xd = np.empty_like(X)
    for s in range(X.shape[1]):
        _, xd[:, s] = R.smoothed_fd4(X[:, s], dt)
    Z = np.concatenate([X, np.asarray(a[:L], dtype=np.float64)[:, None]], axis=1)
    return Z, xd


def ms_gram(x, a, rows, dt, exps):
    """G = sum_p Theta_p^T Theta_p [F, F] and B = sum_p Theta_p^T xdot_p [F, S] over patients with
    >= 5 rows (what insite_gram_ms_f32 returns).  x [N, T, S], a [N, T], rows [N]."""
    F, S = exps.shape[0], x.shape[2]
    G = np.zeros((F, F))
    B = np.zeros((F, S))
    for i in range(x.shape[0]):
        L = int(min(rows[i], x.shape[1]))
        if L < 5:
            continue
        Z, Y = ms_regression(x[i], a[i], L, dt)
        th = R.eval_library(exps, Z)
        G += th.T @ th
        B += th.T @ Y
    return G, B


def ms_gram_vectorized(x, a, dt, exps):
    """Equal-length (rows = T) variant, vectorised over patients (CPU baseline timing)."""
    N, T, S = x.shape
    X = np.asarray(x, dtype=np.float64)
    xs = np.empty_like(X)
    xd = np.empty_like(X)
    for s in range(S):
        xs[:, :, s] = R._stencil5(X[:, :, s].T, R.SAVGOL_5_3).T
        xd[:, :, s] = R._stencil5(xs[:, :, s].T, R.FD4).T / dt
    Z = np.concatenate([X, np.asarray(a, dtype=np.float64)[:, :, None]], axis=2).reshape(N * T, S + 1)
    th = R.eval_library(exps, Z)
    return th.T @ th, th.T @ xd.reshape(N * T, S)


def ms_stlsq(G, B, threshold=THRESHOLD_C3, alpha=ALPHA_C3, max_iter=100, unbias=True):
    """One STLSQ per target on the shared Gram: coef [S, F], mask [S, F], iters [S]."""
    F, S = B.shape
    coef = np.zeros((S, F))
    mask = np.zeros((S, F), dtype=bool)
    iters = np.zeros(S, dtype=np.int64)
    for s in range(S):
        coef[s], mask[s], iters[s] = R.stlsq_gram(G, B[:, s], threshold, alpha, max_iter, unbias)
    return coef, mask, iters


def ms_rollout(y0, a, coef, exps, dt, method="rk4", substeps=1, drop=R.RHS_COEF_EPS):
    """Open-loop rollout of the S-state model: y [N, T, S], y[:, k] = state after interval k with the
    treatment a[:, k] held over it (insite_ref.rollout convention, S-dimensional)."""
    y = np.asarray(y0, dtype=np.float64).copy()
    N, T = a.shape
    out = np.empty((N, T, y.shape[1]))
    for k in range(T):
        ak = a[:, k].astype(np.float64)
        if method in ("euler", "euler5"):
            n_sub = R.STEPS_FOR_DT if method == "euler5" else int(substeps or 1)
            h = dt / n_sub
            for _ in range(n_sub):
                y = y + h * eval_rhs(y, ak, coef, exps, drop)
        elif method == "rk4":
            h = dt / int(substeps or 1)
            for _ in range(int(substeps or 1)):
                k1 = eval_rhs(y, ak, coef, exps, drop)
                k2 = eval_rhs(y + 0.5 * h * k1, ak, coef, exps, drop)
                k3 = eval_rhs(y + 0.5 * h * k2, ak, coef, exps, drop)
                k4 = eval_rhs(y + h * k3, ak, coef, exps, drop)
                y = y + (h / 6.0) * (k1 + 2.0 * k2 + 2.0 * k3 + k4)
        else:
            raise ValueError(method)
        out[:, k] = y
    return out


def ms_pipeline(N=400, T=500, seed=2, dt=DT_C3):
    """C1-sized end-to-end C3 check: cohort -> Gram -> STLSQ; returns (coef, mask, truth)."""
    x, a = c3_cohort(N, T, seed, dt)
    exps = c3_library()
    G, B = ms_gram_vectorized(x, a, dt, exps)
    coef, mask, _ = ms_stlsq(G, B)
    return coef, mask, c3_truth_coef(exps)
