"""CPU restatement of the adaptive RK45 rollout on irregular observation grids — configuration C5 of
BASELINE.json (TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package).

The reference integrates the discovered model per observation interval (``odeint`` over [t_k, t_k+1],
libs_m/ct/src/models/sindy.py:413-424; pkpd/utils.py:68-94) with the treatment held over the interval.
C5 replaces the fixed Euler-5 / RK4 interval map by scipy's adaptive ``solve_ivp(method='RK45')`` with
the reference odeint's tolerances rtol = atol = 1.4e-8 (utils.py:87), on per-patient irregular grids.
The third-party algorithm (scipy 1.15.3, ``scipy/integrate/_ivp/rk.py`` RungeKutta._step_impl, RK45
tableau; ``common.py`` select_initial_step / RMS norm) is restated here for a scalar state:

  * initial step: d0 = |y|/sc, d1 = |f|/sc (sc = atol + |y| rtol), h0 = 1e-6 if d0 < 1e-5 or d1 < 1e-5
    else 0.01 d0/d1, h0 = min(h0, interval); d2 = |f(y + h0 f) - f|/sc/h0; h1 = max(1e-6, 1e-3 h0) if
    d1, d2 <= 1e-15 else (0.01/max(d1, d2))^(1/5); h = min(100 h0, h1, interval);
  * step: h clamped below by 10 ulp(t) and to the interval end; Dormand-Prince stages, 5th-order update,
    error = h (E . K) with K_7 = f(y_new) (FSAL), err = |error| / (atol + max(|y|, |y_new|) rtol);
    accept if err < 1: h *= min(10, 0.9 err^-1/5) (10 if err = 0; capped at 1 after a rejection), else
    h *= max(0.2, 0.9 err^-1/5) and retry.

``rk45_interval`` is pinned against ``scipy.integrate.solve_ivp`` in tests/test_rk45_oracle.py.
"""
from __future__ import annotations

import math

import numpy as np

from . import insite_ref as R

RTOL = 1.4e-8   # reference odeint defaults (pkpd/utils.py:87)
ATOL = 1.4e-8

C = (0.0, 1 / 5, 3 / 10, 4 / 5, 8 / 9, 1.0)
A = ((),
     (1 / 5,),
     (3 / 40, 9 / 40),
     (44 / 45, -56 / 15, 32 / 9),
     (19372 / 6561, -25360 / 2187, 64448 / 6561, -212 / 729),
     (9017 / 3168, -355 / 33, 46732 / 5247, 49 / 176, -5103 / 18656))
B = (35 / 384, 0.0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84)
E = (-71 / 57600, 0.0, 71 / 16695, -71 / 1920, 17253 / 339200, -22 / 525, 1 / 40)
SAFETY, MIN_FACTOR, MAX_FACTOR = 0.9, 0.2, 10.0
ERR_EXP = -1.0 / 5.0


def select_initial_step(f, t0, y0, t1, f0, rtol=RTOL, atol=ATOL):
    interval = abs(t1 - t0)
    if interval == 0.0:
        return 0.0
    scale = atol + abs(y0) * rtol
    d0 = abs(y0 / scale)
    d1 = abs(f0 / scale)
    h0 = 1e-6 if (d0 < 1e-5 or d1 < 1e-5) else 0.01 * d0 / d1
    h0 = min(h0, interval)
    y1 = y0 + h0 * f0
    f1 = f(y1)
    d2 = abs((f1 - f0) / scale) / h0
    if d1 <= 1e-15 and d2 <= 1e-15:
        h1 = max(1e-6, h0 * 1e-3)
    else:
        h1 = (0.01 / max(d1, d2)) ** (1.0 / 5.0)
    return min(100 * h0, h1, interval)


def rk45_interval(f, y, t0, t1, rtol=RTOL, atol=ATOL):
    """Integrate the autonomous scalar ODE y' = f(y) from t0 to t1 (t1 >= t0) as scipy's
    solve_ivp(RK45) does; returns (y(t1), accepted + rejected step attempts)."""
    t = float(t0)
    y = float(y)
    fy = f(y)
    h_abs = select_initial_step(f, t, y, t1, fy, rtol, atol)
    attempts = 0
    while t < t1:
        min_step = 10 * abs(math.nextafter(t, math.inf) - t)
        if h_abs < min_step:
            h_abs = min_step
        rejected = False
        while True:
            h = h_abs
            t_new = t + h
            if t_new > t1:
                t_new = t1
            h = t_new - t
            h_abs = abs(h)
            K = [fy]
            for s in range(1, 6):
                dy = 0.0
                for j, a in enumerate(A[s]):
                    dy += K[j] * a
                K.append(f(y + dy * h))
            acc = 0.0
            for j in range(6):
                acc += K[j] * B[j]
            y_new = y + h * acc
            f_new = f(y_new)
            K.append(f_new)
            scale = atol + max(abs(y), abs(y_new)) * rtol
            e = 0.0
            for j in range(7):
                e += K[j] * E[j]
            err = abs(e * h / scale)
            attempts += 1
            if err < 1:
                factor = MAX_FACTOR if err == 0 else min(MAX_FACTOR, SAFETY * err ** ERR_EXP)
                if rejected:
                    factor = min(1.0, factor)
                h_abs *= factor
                break
            h_abs *= max(MIN_FACTOR, SAFETY * err ** ERR_EXP)
            rejected = True
        t, y, fy = t_new, y_new, f_new
    return y, attempts


def patient_rates(u, coef, exps, drop=R.RHS_COEF_EPS):
    """(alpha[A], beta[A]) of f_a(y) = alpha_a + beta_a y for one patient: the library is affine in the
    state (INSITE_MAX_STATE_DEGREE 1); terms with |c| <= drop are dropped (utils.py:388)."""
    A_ = coef.shape[0]
    al = np.zeros(A_)
    be = np.zeros(A_)
    for a in range(A_):
        for j, e in enumerate(exps):
            c = coef[a, j]
            if abs(c) <= drop:
                continue
            m = 1.0
            for i in range(1, e.shape[0]):
                for _ in range(int(e[i])):
                    m *= u[i - 1]
            if e[0] == 0:
                al[a] += c * m
            else:
                be[a] += c * m
    return al, be


def rollout_rk45(y0, u, arm, t_obs, n_obs, coef, exps, rtol=RTOL, atol=ATOL):
    """Per patient p and interval k < n_obs[p] - 1: y <- RK45 of f_{arm[p, k]} over [t_obs[p, k],
    t_obs[p, k + 1]].  Returns y [N, Tmax] (state after interval k; NaN past the patient's grid) and
    the step attempts per patient."""
    N, Tm = t_obs.shape
    out = np.full((N, Tm), np.nan)
    steps = np.zeros(N, dtype=np.int64)
    for p in range(N):
        al, be = patient_rates(u[p], coef, exps)
        y = float(y0[p])
        for k in range(int(n_obs[p]) - 1):
            a = int(arm[p, k])
            y, n = rk45_interval(lambda v, a=a: al[a] + be[a] * v, y, t_obs[p, k], t_obs[p, k + 1], rtol, atol)
            steps[p] += n
            out[p, k] = y
    return out, steps


def irregular_grid(N, rng, t_max=R.MAX_TIME_HORIZON, n_min=20, n_max=60):
    """C5 observation grids: T_p ~ U{n_min..n_max}, t_0 = 0 and T_p - 1 sorted U(0, t_max) times."""
    n_obs = rng.integers(n_min, n_max + 1, N).astype(np.int32)
    Tm = int(n_max)
    t = np.full((N, Tm), np.nan)
    for p in range(N):
        t[p, 0] = 0.0
        t[p, 1:n_obs[p]] = np.sort(rng.uniform(0.0, t_max, n_obs[p] - 1))
    return t, n_obs
