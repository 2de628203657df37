"""CPU restatement of the INSITE per-patient refinement — TEST INFRASTRUCTURE ONLY
(imported by tests/ and bench.py's cpu_baseline leg, never by the product package).

Reference: ``SINDY._get_fine_tuned_predictions`` / ``f_to_min_func`` / ``predict_with_reduced_coefs``
(libs_m/ct/src/models/sindy.py:433-715, 767-794).  Per patient with sequence_length > tau:

  mask    = |c0| > 1e-3                                  (coef_sparse_mask, :587)
  preds   = Euler-5 scan of sum_j c_aj Theta_j(y, u) from V[0] under the patient's per-step arms
  mse(c)  = sum_{k < sl - tau} (V[k+1] - preds[k])^2 / #      (create_mask, pkpd/utils.py:367-370; :781-792)
  f(c)    = mse(c * mask) / (2.5 mse(c0)) + lam * mean((c0 - c)^2)       (norm_const = start_res * 2.5, :614)
  c*      = jax.scipy.optimize.minimize(f, c0, method='BFGS', tol=1e-12)  (:627); status 3 -> keep c0 (:628-631)
  output  = preds(c*) over the whole row                                  (:668)

Pinned against REFERENCE-HELD OUTPUTS: on the reference's own EQ_4_A..D cohorts (oracle/ref_cohort.py)
the refined one-step and tau-step metrics reproduce the published INSITE runs
(results/2_main_table/final_with_insite.txt:2387-2402) to <= 1e-10 relative (EQ_4_A: 7e-14) — 283k
refinements through this BFGS / line-search / zoom restatement — PROVIDED rows whose zoom fails
(status 3) keep their BFGS iterate.  With the status-3 revert of sindy.py:628-631 applied, the noisy
cohorts miss the log by 1e-3 (EQ_4_B/C) to 3e-1 (EQ_4_D, 430 of 11,600 one-step rows revert): those
rows sit at rounding-level flatness of the objective (mse divided by 2.5 x its tiny start value),
where our arithmetic exhausts the 30 zoom iterations and jax's evidently did not.  The default
``revert_on_zoom_fail=False`` therefore follows the published outputs; True is the literal code.

The minimiser is a third-party algorithm: jax (unpinned; a transitive dependency of sympy2jax,
setup/requirements.txt) ``jax/_src/scipy/optimize/{minimize,bfgs,line_search}.py``, restated here:
``minimize`` passes no tolerance to ``minimize_bfgs`` (gtol = 1e-5 on the inf-norm of the gradient,
maxiter = 200 * size(x0), line_search maxiter = 10), BFGS with H0 = I and the inverse update
H <- (I - rho s y^T) H (I - rho y s^T) + rho s s^T (kept when rho is not finite); strong-Wolfe line search
(c1 = 1e-4, c2 = 0.9, first trial min(1, 1.01 * 2 (f_k - f_{k-1}) / phi'(0)), then doubling) with the
cubic / quadratic / bisection zoom (delta1 = 0.2, delta2 = 0.1, dalpha threshold 1e-10, and jax's
``failed | j >= 30`` written without parentheses, i.e. (failed | j) >= 30).  Status: 0 converged, 1
maxiter, 2 + line-search status (1 zoom failed, 3 line-search maxiter).  Without jax this restatement
is **parity unpinned** against the reference; tests pin the objective/gradient (finite differences), the
minimiser (scipy.optimize.minimize BFGS reaches the same optimum) and the GPU kernel (same algorithm).

Only the masked-in coefficients move: inactive ones have zero data gradient and start at c0, so the
penalty gradient is zero and BFGS (H0 = I) keeps its inverse Hessian block-diagonal — the search runs
in the m-dimensional active subspace with identical arithmetic (the mean is still over all A*F).
"""
from __future__ import annotations

import numpy as np

from . import insite_ref as R

C1, C2 = 1e-4, 0.9
GTOL = 1e-5
LS_MAXITER = 10
MASK_EPS = 1e-3


def coef_terms(c0, exps, n_inputs=0):
    """Per flat coefficient q of the global model c0 [A, F]: (arm mask, state exponent, static exponents).

    Separate models (n_inputs = 0, sindy.py:457-467, 489-499, 523-533): coefficient (a, j) acts on arm a
    only, mask 1 << a.  The joint model (n_inputs > 0, c0 [1, F], library inputs (x0, in_1..in_n, statics),
    sindy.py:469-483, 503-517, 537-551): the per-step treatments are binary library inputs, so column j,
    x^e in^tau m(u), contributes m(u) x^e on every treatment combination c (arm = bit code of the step's
    treatments) whose bits cover tau's inputs -- the fold of ``insite_amd.sindy.SINDY._fold_joint``."""
    A, F = c0.shape
    out = []
    for a in range(A):
        for j in range(F):
            e = exps[j]
            if n_inputs:
                tin = sum(1 << i for i in range(n_inputs) if e[1 + i] > 0)
                mask = sum(1 << c for c in range(1 << n_inputs) if (tin & ~c) == 0)
                ue = tuple(int(v) for v in e[1 + n_inputs:])
            else:
                mask, ue = 1 << a, tuple(int(v) for v in e[1:])
            out.append((mask, int(e[0]), ue))
    return out


def n_arms_of(c0, n_inputs=0):
    return (1 << n_inputs) if n_inputs else c0.shape[0]


def active_terms(c0, exps, n_inputs=0):
    """Active coefficients (|c0| > 1e-3): list of (flat index, arm mask, state exponent, static exponents)."""
    terms = coef_terms(c0, exps, n_inputs)
    return [(q, *terms[q]) for q in range(c0.size) if abs(c0.flat[q]) > MASK_EPS]


def static_monomial(u, ue):
    m = 1.0
    for i, k in enumerate(ue):
        for _ in range(int(k)):
            m *= u[i]
    return m


def monomials(u, exps):
    m = np.ones(exps.shape[0])
    for j, e in enumerate(exps):
        for i in range(1, e.shape[0]):
            for _ in range(int(e[i])):
                m[j] *= u[i - 1]
    return m


def _poly(g, y):
    """sum_e g[e] y^e by Horner (the state-polynomial RHS of one arm)."""
    f = g[-1]
    for e in range(len(g) - 2, -1, -1):
        f = g[e] + f * y
    return f


def _dpoly(g, y):
    """d/dy sum_e g[e] y^e by Horner."""
    D = len(g) - 1
    f = D * g[D]
    for e in range(D - 1, 0, -1):
        f = e * g[e] + f * y
    return f


class PatientProblem:
    """f(c_active) and its gradient for one patient: V [T'] unscaled observations, arms [T'] per step (the
    arm index, or the treatment combination's bit code for the joint model), K = min(sl - tau, T' - 1)
    loss terms.  The RHS of arm a is the state polynomial sum_e gamma_{a,e} y^e, gamma_{a,e} = sum over the
    active coefficients q with arm a in mask_q and exponent e of c_q m_q(u); degree 1 is the affine
    (alpha_a, beta_a) of the paper's libraries, degree 4 the ABLATION_MORE_COMPLEX_BASIS_FUNCTIONS library."""

    def __init__(self, V, arms, u, c0, exps, K, dt, lam, substeps=R.STEPS_FOR_DT, n_inputs=0):
        self.V = np.asarray(V, dtype=np.float64)
        self.arms = np.asarray(arms, dtype=np.int64)
        self.terms = active_terms(c0, exps, n_inputs)
        self.mono = np.array([static_monomial(u, t[3]) for t in self.terms])
        self.c0 = np.array([c0.flat[t[0]] for t in self.terms])
        self.n_total = c0.size
        self.K = int(K)
        self.h = dt / substeps
        self.sub = substeps
        self.lam = lam
        self.norm = 1.0
        self.A = n_arms_of(c0, n_inputs)
        self.D = max(1, int(np.max(exps[:, 0])))

    def rates(self, c):
        gam = np.zeros((self.A, self.D + 1))
        for ci, mi, (_, mask, ex, _) in zip(c, self.mono, self.terms):
            for a in range(self.A):
                if (mask >> a) & 1:
                    gam[a, ex] += ci * mi
        return gam

    def mse_and_grad(self, c):
        """Euler-5 rollout with forward sensitivities d y / d gamma_{a,e}."""
        gam = self.rates(c)
        A, D = self.A, self.D
        y = self.V[0]
        d = np.zeros((A, D + 1))
        L = 0.0
        gG = np.zeros((A, D + 1))
        h = self.h
        for k in range(self.K):
            a = self.arms[k]
            g = gam[a]
            for _ in range(self.sub):
                if D == 1:
                    hb = h * g[1]
                    nd = d + hb * d
                    nd[a, 0] += h
                    nd[a, 1] += h * y
                    y = y + h * (g[0] + g[1] * y)
                else:
                    hf = h * _dpoly(g, y)
                    nd = d + hf * d
                    ye = 1.0
                    for e in range(D + 1):
                        nd[a, e] += h * ye
                        ye *= y
                    y = y + h * _poly(g, y)
                d = nd
            r = self.V[k + 1] - y
            L += r * r
            gG += -2.0 * r * d
        return L / self.K, gG / self.K

    def value_and_grad(self, c):
        L, gG = self.mse_and_grad(c)
        f = L / self.norm + self.lam * np.sum((self.c0 - c) ** 2) / self.n_total
        g = np.empty_like(c)
        for i, (_, mask, ex, _) in enumerate(self.terms):
            gd = 0.0
            for a in range(self.A):
                if (mask >> a) & 1:
                    gd += gG[a, ex]
            g[i] = gd * self.mono[i] / self.norm
        g += 2.0 * self.lam * (c - self.c0) / self.n_total
        return f, g


# ------------------------------------------------------------------------------------------------
# jax.scipy.optimize BFGS + line search (restated)
# ------------------------------------------------------------------------------------------------
def _cubicmin(a, fa, fpa, b, fb, c, fc):
    C = fpa
    db = b - a
    dc = c - a
    denom = (db * dc) ** 2 * (db - dc)
    d1 = np.array([[dc ** 2, -db ** 2], [-dc ** 3, db ** 3]])
    d2 = np.array([fb - fa - C * db, fc - fa - C * dc])
    with np.errstate(all="ignore"):
        A, B = (d1 @ d2) / denom
        radical = B * B - 3.0 * A * C
        return a + (-B + np.sqrt(radical)) / (3.0 * A)


def _quadmin(a, fa, fpa, b, fb):
    D = fa
    C = fpa
    db = b - 1.0 * a
    with np.errstate(all="ignore"):
        B = (fb - D - C * db) / (db ** 2)
        return a - C / (2.0 * B)


def _zoom(phi_fn, wolfe_one, wolfe_two, a_lo, phi_lo, dphi_lo, a_hi, phi_hi, dphi_hi, g_0):
    st = dict(done=False, failed=False, j=0, a_lo=a_lo, phi_lo=phi_lo, dphi_lo=dphi_lo, a_hi=a_hi, phi_hi=phi_hi,
              dphi_hi=dphi_hi, a_rec=(a_lo + a_hi) / 2.0, phi_rec=(phi_lo + phi_hi) / 2.0, a_star=1.0,
              phi_star=phi_lo, dphi_star=dphi_lo, g_star=g_0, nfev=0)
    delta1, delta2 = 0.2, 0.1
    while (not st["done"]) and (not st["failed"]):
        dalpha = st["a_hi"] - st["a_lo"]
        a = min(st["a_hi"], st["a_lo"])
        b = max(st["a_hi"], st["a_lo"])
        cchk = delta1 * dalpha
        qchk = delta2 * dalpha
        st["failed"] = st["failed"] or (dalpha <= 1e-10)
        a_cub = _cubicmin(st["a_lo"], st["phi_lo"], st["dphi_lo"], st["a_hi"], st["phi_hi"], st["a_rec"], st["phi_rec"])
        use_cubic = (st["j"] > 0) and (a_cub > a + cchk) and (a_cub < b - cchk)
        a_quad = _quadmin(st["a_lo"], st["phi_lo"], st["dphi_lo"], st["a_hi"], st["phi_hi"])
        use_quad = (not use_cubic) and (a_quad > a + qchk) and (a_quad < b - qchk)
        use_bis = (not use_cubic) and (not use_quad)
        a_j = st["a_rec"]
        if use_cubic:
            a_j = a_cub
        if use_quad:
            a_j = a_quad
        if use_bis:
            a_j = (st["a_lo"] + st["a_hi"]) / 2.0
        phi_j, dphi_j, g_j = phi_fn(a_j)
        st["nfev"] += 1
        hi_to_j = wolfe_one(a_j, phi_j) or (phi_j >= st["phi_lo"])
        star_to_j = wolfe_two(dphi_j) and (not hi_to_j)
        hi_to_lo = (dphi_j * (st["a_hi"] - st["a_lo"]) >= 0.0) and (not hi_to_j) and (not star_to_j)
        lo_to_j = (not hi_to_j) and (not star_to_j)
        if hi_to_j:
            st.update(a_hi=a_j, phi_hi=phi_j, dphi_hi=dphi_j, a_rec=st["a_hi"], phi_rec=st["phi_hi"])
        st["done"] = star_to_j or st["done"]
        if star_to_j:
            st.update(a_star=a_j, phi_star=phi_j, dphi_star=dphi_j, g_star=g_j)
        if hi_to_lo:
            st.update(a_hi=st["a_lo"], phi_hi=st["phi_lo"], dphi_hi=st["dphi_lo"], a_rec=st["a_hi"],
                      phi_rec=st["phi_hi"])
        if lo_to_j:
            st.update(a_lo=a_j, phi_lo=phi_j, dphi_lo=dphi_j, a_rec=st["a_lo"], phi_rec=st["phi_lo"])
        st["j"] += 1
        st["failed"] = (int(st["failed"]) | st["j"]) >= 30    # jax: failed | j >= 30 (no parentheses)
    return st


def line_search(fg, xk, pk, old_fval, old_old_fval, gfk, maxiter=LS_MAXITER):
    def phi_fn(t):
        f, g = fg(xk + t * pk)
        return f, float(g @ pk), g

    phi_0 = old_fval
    dphi_0 = float(gfk @ pk)
    cand = 1.01 * 2 * (phi_0 - old_old_fval) / dphi_0
    start = 1.0 if cand > 1 else cand

    def wolfe_one(a_i, phi_i):
        return phi_i > phi_0 + C1 * a_i * dphi_0

    def wolfe_two(dphi_i):
        return abs(dphi_i) <= -C2 * dphi_0

    st = dict(done=False, failed=False, i=1, a_i1=0.0, phi_i1=phi_0, dphi_i1=dphi_0, nfev=0, a_star=0.0,
              phi_star=phi_0, dphi_star=dphi_0, g_star=gfk)
    while (not st["done"]) and (st["i"] <= maxiter) and (not st["failed"]):
        a_i = start if st["i"] == 1 else st["a_i1"] * 2.0
        phi_i, dphi_i, g_i = phi_fn(a_i)
        st["nfev"] += 1
        s_z1 = wolfe_one(a_i, phi_i) or ((phi_i >= st["phi_i1"]) and (st["i"] > 1))
        s_i = wolfe_two(dphi_i) and (not s_z1)
        s_z2 = (dphi_i >= 0.0) and (not s_z1) and (not s_i)
        if s_z1:
            z = _zoom(phi_fn, wolfe_one, wolfe_two, st["a_i1"], st["phi_i1"], st["dphi_i1"], a_i, phi_i, dphi_i, gfk)
            st["nfev"] += z["nfev"]
            st["failed"] = st["failed"] or z["failed"]
            st.update(a_star=z["a_star"], phi_star=z["phi_star"], dphi_star=z["dphi_star"], g_star=z["g_star"])
        if s_i:
            st.update(a_star=a_i, phi_star=phi_i, dphi_star=dphi_i, g_star=g_i)
        if s_z2:
            z = _zoom(phi_fn, wolfe_one, wolfe_two, a_i, phi_i, dphi_i, st["a_i1"], st["phi_i1"], st["dphi_i1"], gfk)
            st["nfev"] += z["nfev"]
            st["failed"] = st["failed"] or z["failed"]
            st.update(a_star=z["a_star"], phi_star=z["phi_star"], dphi_star=z["dphi_star"], g_star=z["g_star"])
        st["done"] = s_z1 or st["done"] or s_i or s_z2
        st.update(i=st["i"] + 1, a_i1=a_i, phi_i1=phi_i, dphi_i1=dphi_i)
    status = 1 if st["failed"] else (3 if st["i"] > maxiter else 0)
    return dict(failed=st["failed"] or not st["done"], a_k=st["a_star"], f_k=st["phi_star"], g_k=st["g_star"],
                status=status, nfev=st["nfev"])


def minimize_bfgs(fg, x0, maxiter, gtol=GTOL, ls_maxiter=LS_MAXITER):
    """jax minimize_bfgs (norm = inf): returns (x, f, status, iterations, function evaluations).
    ``gtol`` / ``maxiter`` / ``ls_maxiter`` are jax's ``minimize_bfgs`` options (defaults 1e-5, 200 * size,
    10); the reference passes none of them (sindy.py:627), they are exposed for the stopping-control sweep
    (tools/insite_stop_sweep.py)."""
    d = x0.size
    H = np.eye(d)
    f, g = fg(x0)
    x = x0.copy()
    converged = np.max(np.abs(g)) < gtol if d else True
    failed = False
    k = 0
    nfev = 1
    old_old = f + np.linalg.norm(g) / 2
    ls_status = 0
    while (not converged) and (not failed) and k < maxiter:
        p = -(H @ g)
        ls = line_search(fg, x, p, f, old_old, g, maxiter=ls_maxiter)
        nfev += ls["nfev"]
        failed = ls["failed"]
        ls_status = ls["status"]
        s = ls["a_k"] * p
        x_new = x + s
        f_new, g_new = ls["f_k"], ls["g_k"]
        y = g_new - g
        with np.errstate(all="ignore"):
            rho = np.float64(1.0) / np.float64(y @ s)
        if np.isfinite(rho):
            w = np.eye(d) - rho * np.outer(s, y)
            H = w @ H @ w.T + rho * np.outer(s, s)
        converged = np.max(np.abs(g_new)) < gtol
        old_old = f
        x, f, g = x_new, f_new, g_new
        k += 1
    status = 0 if converged else (1 if k == maxiter else (2 + ls_status if failed else -1))
    return x, f, status, k, nfev


def euler5_rollout(V0, arms, u, coef, exps, dt, T, n_inputs=0):
    """predict_with_reduced_coefs (sindy.py:767-778): Euler-5 scan with every coefficient (no RHS drop);
    arms [T] per-step arm index (joint model: treatment bit code)."""
    terms = coef_terms(coef, exps, n_inputs)
    A = n_arms_of(coef, n_inputs)
    D = max(1, int(np.max(exps[:, 0])))
    gam = np.zeros((A, D + 1))
    for q, (mask, ex, ue) in enumerate(terms):
        for a in range(A):
            if (mask >> a) & 1:
                gam[a, ex] += coef.flat[q] * static_monomial(u, ue)
    y = float(V0)
    out = np.empty(T)
    h = dt / R.STEPS_FOR_DT
    for k in range(T):
        g = gam[int(arms[k])]
        for _ in range(R.STEPS_FOR_DT):
            y = y + h * (g[0] + g[1] * y) if D == 1 else y + h * _poly(g, y)
        out[k] = y
    return out


def refine_patient(V, arms, u, sl, c0, exps, dt, lam, tau, revert_on_zoom_fail=False, n_inputs=0,
                   gtol=GTOL, maxiter=None, ls_maxiter=LS_MAXITER, revert_statuses=None):
    """One patient of ``simulate_cancer_volume_with_fine_tuning`` (sindy.py:570-668).  Returns
    (preds [T'], refined coefficients [A, F], status, iterations); status -1 = skipped (sl <= tau).
    ``revert_on_zoom_fail``: status 3 keeps c0 (sindy.py:628-631); default False = the published runs
    (module docstring).  ``n_inputs`` > 0: the joint model (c0 [1, F], arms = treatment bit codes).
    ``gtol`` / ``maxiter`` (default 200 * c0.size, jax's) / ``ls_maxiter`` / ``revert_statuses`` (a set of
    statuses that keep c0, overriding ``revert_on_zoom_fail``) exist for the stopping-control sweep only."""
    T = V.shape[0]
    c0 = np.asarray(c0, dtype=np.float64)
    if sl <= tau:
        return euler5_rollout(V[0], arms, u, c0, exps, dt, T, n_inputs), c0.copy(), -1, 0
    K = min(int(sl) - tau, T - 1)
    pb = PatientProblem(V, arms, u, c0, exps, K, dt, lam, n_inputs=n_inputs)
    start, _ = pb.value_and_grad(pb.c0)          # norm_const = 1, penalty 0 at c0
    pb.norm = start * 2.5
    x, f, status, k, _ = minimize_bfgs(pb.value_and_grad, pb.c0.copy(),
                                       maxiter=200 * c0.size if maxiter is None else int(maxiter),
                                       gtol=gtol, ls_maxiter=ls_maxiter)
    c = c0.copy()
    revert = (status in revert_statuses) if revert_statuses is not None else (status == 3 and revert_on_zoom_fail)
    if not revert:
        for xi, t in zip(x, pb.terms):
            c.flat[t[0]] = xi
    return euler5_rollout(V[0], arms, u, c, exps, dt, T, n_inputs), c, status, k
