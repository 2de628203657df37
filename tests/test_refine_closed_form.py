"""The closed-form step map of the INSITE objective scans (INSITE_REFINE_CF, csrc/insite_refine.hip cf_arm) against
the sub-step recurrences it replaces (oracle/insite_refine_ref.py PatientProblem.mse_and_grad, the reference's
odeint Euler sub-steps, pkpd/utils.py:68-79): y <- y + h (g0 + g1 y) n times, with the forward sensitivities
d/dg_{a,0} <- d (1 + h g1) + h [a active], d/dg_{a,1} <- d (1 + h g1) + h y [a active].  CPU only (numpy)."""
import numpy as np
import pytest


def cf_arm(g0, g1, h, n):
    """The kernel's per-arm constants (P, B, hS, C1, C2), same loop and operation order."""
    q = 1.0 + h * g1
    pw, S, Cs, qn1 = 1.0, 0.0, 0.0, 1.0
    for j in range(n):
        if j + 1 < n:
            Cs = (j + 1) * pw + Cs
        S += pw
        qn1 = pw
        pw *= q
    return pw, h * g0 * S, h * S, n * h * qn1, h * h * g0 * Cs


def substeps(y, d0, d1, e0, e1, g0, g1, h, n):
    """n Euler sub-steps on the active arm: (y, its two tangents d0 / d1, another arm's tangents e0 / e1)."""
    for _ in range(n):
        hb = h * g1
        d0, d1 = d0 + hb * d0 + h, d1 + hb * d1 + h * y
        e0, e1 = e0 + hb * e0, e1 + hb * e1
        y = y + h * (g0 + g1 * y)
    return y, d0, d1, e0, e1


@pytest.mark.parametrize("n", [1, 2, 5, 7])
def test_closed_form_step_equals_substeps(n):
    rng = np.random.default_rng(n)
    worst = 0.0
    for _ in range(2000):
        g0, g1 = rng.normal(0.0, 2.0), rng.normal(-0.5, 1.0)
        h = rng.uniform(1e-3, 0.05)
        y, d0, d1, e0, e1 = rng.normal(size=5) * np.array([5.0, 1.0, 3.0, 1.0, 3.0])
        want = substeps(y, d0, d1, e0, e1, g0, g1, h, n)
        P, B, hS, C1, C2 = cf_arm(g0, g1, h, n)
        got = (P * y + B, P * d0 + hS, P * d1 + (C1 * y + C2), P * e0, P * e1)
        for a, b in zip(got, want):
            worst = max(worst, abs(a - b) / max(1.0, abs(b)))
    assert worst < 1e-12, worst


def test_closed_form_scan_gradient_matches_oracle():
    """A whole objective and gradient through the closed form equal the oracle's sub-step scan (the restatement the
    GPU parity tests compare against) to rounding."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import insite_refine_ref as RR

    rng = np.random.default_rng(3)
    T, K, n, dt = 40, 30, 5, 10.0 / 60
    h = dt / n
    exps = np.array([[0, 0], [1, 0], [0, 1], [1, 1]])  # 1, x0, u0, x0 u0 (one static)
    c0 = np.array([[0.4, -0.3, 0.2, -0.1], [0.1, -0.6, 0.3, 0.05]])
    u = np.array([1.3])
    arms = (np.arange(T) >= 17).astype(np.int64)  # one switch inside the window
    V = 5.0 + rng.normal(0.0, 0.3, T)
    pb = RR.PatientProblem(V, arms, u, c0, exps, K, dt, 10.0, substeps=n)
    c = pb.c0 * (1.0 + 0.05 * rng.normal(size=pb.c0.size))
    L_ref, gG_ref = pb.mse_and_grad(c)
    gam = pb.rates(c)
    y = V[0]
    d = np.zeros((2, 2))
    L, gG = 0.0, np.zeros((2, 2))
    cf = [cf_arm(gam[a, 0], gam[a, 1], h, n) for a in range(2)]
    for k in range(K):
        a = arms[k]
        P, B, hS, C1, C2 = cf[a]
        add1 = C1 * y + C2
        for b in range(2):
            d[b, 0] = P * d[b, 0] + (hS if b == a else 0.0)
            d[b, 1] = P * d[b, 1] + (add1 if b == a else 0.0)
        y = P * y + B
        r = V[k + 1] - y
        L += r * r
        gG += -2.0 * r * d
    L, gG = L / K, gG / K
    assert abs(L - L_ref) <= 1e-12 * abs(L_ref)
    assert np.max(np.abs(gG - gG_ref)) <= 1e-11 * max(1.0, np.max(np.abs(gG_ref)))
