"""segments_ref — CPU restatement of the cancer_sim / EQ_5 discovery path.

TEST INFRASTRUCTURE ONLY (same rules as ``insite_ref``): imported by ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg, never by the product.

What it restates (reference file:line):

* ``process_sindy_training_data`` for ``Datasets.CANCER_SIM`` / ``EQ_5``
  (``libs_m/ct/src/data/pkpd/utils.py:433-462``): every patient's series is cut into
  treatment-constant segments.  Walking ``i = 0 .. seq_len-1``: when ``treatments[i]`` differs
  from the running segment's last treatment, the running segment is closed with one more sample
  ``cancer[i]`` (carrying the previous treatment: consecutive segments share their boundary
  sample) and a new one starts at ``cancer[i]``; at ``i = seq_len-1`` the running segment is closed
  with ``cancer[seq_len]``.  Every segment therefore holds >= 2 samples.
* ``process_dataset_into_de_format`` (``utils.py:607-637``): ``sequence_lengths_offset = 0``;
  segment arm = ``argmax(action.mean(0))`` (the one-hot's index: a segment's treatment rows are
  identical), four per-arm trajectory lists.
* ``SINDY.fit`` (``libs_m/ct/src/models/sindy.py:193-216``): one pysindy ``SINDy`` per arm with
  ``FiniteDifference(is_uniform=True, order=1)`` (``use_smoothed_finite_difference: false`` in
  ``config/backbone/{sindy,insite}.yaml:16``) or ``SmoothedFiniteDifference(savgol window 2,
  polyorder 1)`` when that flag is set, ``PolynomialLibrary(degree=2, interaction_only=True)``
  over ``[x0, statics]`` (cancer_sim: 1 static -> F = 4 ``1, x0, u0, x0 u0``; EQ_5: 2 statics ->
  F = 7), ``STLSQ(threshold, alpha, max_iter=100)`` on the concatenated segments of each arm.
* the 4-arm RHS ``lax.switch(argmax(treatment), ...)`` (``sindy.py:289-312``) and
  ``global_equation_string`` with four ``Treatment a:`` parts (``:295``).

Pins (tests/test_segments_oracle.py): the index-form segment walk equals a literal transcription
of the reference loop on one-hot treatment arrays (ragged lengths, switches at the first/last step,
single-arm patients); FD order 1 is pysindy 1.7's uniform ``FiniteDifference(order=1)`` (forward
difference, backward at the last sample — ``insite_ref.fd_order1``); the savgol(2, 1) smoother is
checked against ``scipy.signal.savgol_filter`` itself; STLSQ is ``insite_ref.stlsq`` (pinned against
sklearn's ridge and numpy lstsq there); the Gram form equals the row form; the planted 4-arm system
of ``synthetic_cohort`` is recovered (support) from noise-free data.  pysindy itself is absent, so the
FD-order-1 stencil choice is "parity unpinned" beyond the published 1.7 stencil rule (as for FD4).
The cancer_sim / EQ_5 *simulators* (``data/cancer_sim``, ``data/continuous/continuous.py``) are
not on the path: ``synthetic_cohort`` is a build-defined 4-arm cohort with the same layout.
"""
from __future__ import annotations

import numpy as np

from . import insite_ref as R


# --------------------------------------------------------------------------------------
# F4 — treatment-constant segmentation (utils.py:433-462, 607-637)
# --------------------------------------------------------------------------------------
def split_segments_onehot(treatments, cancer, static, seq_len):
    """Literal restatement of the reference walk (utils.py:434-462) on one-hot
    ``treatments[>= seq_len, A]``, ``cancer[>= seq_len + 1]`` and ``static[>= seq_len + 1, U]``.
    Returns ``(treatments_l_all, outputs_l_all, static_l_all)``."""
    t_all, o_all, s_all = [], [], []
    t_l, o_l, s_l = [], [], []
    for i in range(int(seq_len)):
        tr = treatments[i]
        if len(t_l) >= 1 and (tr != t_l[-1]).any():
            t_l.append(t_l[-1])
            o_l.append(cancer[i])
            s_l.append(static[i])
            t_all.append(np.stack(t_l))
            o_all.append(np.stack(o_l).reshape(-1, 1))
            s_all.append(np.stack(s_l))
            t_l, o_l, s_l = [tr], [cancer[i]], [static[i]]
        else:
            t_l.append(tr)
            o_l.append(cancer[i])
            s_l.append(static[i])
        if i == seq_len - 1:
            t_l.append(tr)
            o_l.append(cancer[i + 1])
            s_l.append(static[i + 1])
            t_all.append(np.stack(t_l))
            o_all.append(np.stack(o_l).reshape(-1, 1))
            s_all.append(np.stack(s_l))
    return t_all, o_all, s_all


def segment_bounds(arm_idx, seq_len):
    """Index form of the same walk for an integer arm sequence ``arm_idx[>= seq_len]``:
    list of ``(arm, start, end)``, the segment holding samples ``start .. end`` inclusive."""
    out = []
    s = 0
    L = int(seq_len)
    for i in range(1, L):
        if arm_idx[i] != arm_idx[i - 1]:
            out.append((int(arm_idx[s]), s, i))
            s = i
    if L >= 1:
        out.append((int(arm_idx[s]), s, L))
    return out


def de_segments(x, u, arm_steps, seq_len, n_arms=4):
    """Per-arm trajectory lists ``(X_a, U_a)`` of ``process_dataset_into_de_format``
    (utils.py:607-637): x[N, >= max(seq_len)+1], u[N, U] (statics, constant over time),
    arm_steps[N, >= max(seq_len)] integer arms (argmax of the one-hot, utils.py:624)."""
    X = [[] for _ in range(n_arms)]
    Ul = [[] for _ in range(n_arms)]
    for i in range(x.shape[0]):
        for a, s, e in segment_bounds(arm_steps[i], seq_len[i]):
            m = e - s + 1
            X[a].append(x[i, s:e + 1].reshape(-1, 1))
            Ul[a].append(np.repeat(u[i][None, :], m, axis=0))
    return X, Ul


# --------------------------------------------------------------------------------------
# derivative estimators of the F4 path (sindy.py:195-203)
# --------------------------------------------------------------------------------------
def savgol_2_1(x):
    """``scipy.signal.savgol_filter(x, window_length=2, polyorder=1)`` (mode 'interp'):
    ``savgol_coeffs(2, 1)`` = [1/2, 1/2] about pos = 0.5, which ``convolve1d`` (even-length weights)
    applies as y[i] = (x[i] + x[i+1]) / 2; the ``window_length // 2 = 1`` sample at either end is
    replaced by the degree-1 polyfit of the first / last two samples, y[0] = x[0], y[-1] = x[-1]
    (to rounding).  Pinned against scipy in tests/test_segments_oracle.py."""
    x = np.asarray(x, dtype=np.float64)
    y = np.empty_like(x)
    y[:-1] = 0.5 * (x[:-1] + x[1:])
    y[0] = x[0]
    y[-1] = x[-1]
    return y


def derivative(x, dt, fd="order1"):
    """(library input, x_dot) of one segment."""
    if fd == "order1":
        return np.asarray(x, dtype=np.float64), R.fd_order1(x, dt)
    if fd == "smoothed1":   # the smoothing feeds x_dot only; the library takes the raw x (insite_ref.smoothed_fd4)
        return np.asarray(x, dtype=np.float64), R.fd_order1(savgol_2_1(x), dt)
    raise ValueError(fd)


# --------------------------------------------------------------------------------------
# SINDy.fit per arm (sindy.py:193-216) — row form and Gram form
# --------------------------------------------------------------------------------------
def build_rows(X_list, U_list, dt, fd="order1"):
    Z, Y = [], []
    for Xs, Us in zip(X_list, U_list):
        xs, xd = derivative(Xs[:, 0], dt, fd)
        Z.append(np.concatenate([xs[:, None], Us], axis=1))
        Y.append(xd)
    if not Z:
        return None, None
    return np.concatenate(Z, axis=0), np.concatenate(Y, axis=0)


def sindy_fit_segments(x, u, arm_steps, seq_len, dt, threshold=1e-3, alpha=0.5, max_iter=100, fd="order1",
                       n_arms=4, degree=2, interaction_only=True):
    """Row-form restatement (what the four pysindy fits compute): returns coef[A, F], ind[A, F],
    iters[A], exps.  An arm without segments raises (pysindy cannot fit an empty list)."""
    exps = R.poly_library(1 + u.shape[1], degree, interaction_only)    # degree 4: sindy.py:185-186
    X, Ul = de_segments(x, u, arm_steps, seq_len, n_arms)
    F = exps.shape[0]
    coef = np.zeros((n_arms, F))
    ind = np.zeros((n_arms, F), dtype=bool)
    iters = np.zeros(n_arms, dtype=np.int64)
    for a in range(n_arms):
        if not X[a]:
            raise ValueError(f"arm {a} has no treatment segments")
        Z, Y = build_rows(X[a], Ul[a], dt, fd)
        coef[a], ind[a], iters[a] = R.stlsq(R.eval_library(exps, Z), Y, threshold, alpha, max_iter)
    return coef, ind, iters, exps


def gram_segments(x, u, arm_steps, seq_len, dt, exps, n_arms=4, fd="order1"):
    """G[A, F, F], b[A, F] and per-arm sample counts — what ``insite_gram_segments_f64`` returns."""
    F = exps.shape[0]
    G = np.zeros((n_arms, F, F))
    b = np.zeros((n_arms, F))
    cnt = np.zeros(n_arms, dtype=np.int64)
    X, Ul = de_segments(x, u, arm_steps, seq_len, n_arms)
    for a in range(n_arms):
        for Xs, Us in zip(X[a], Ul[a]):
            Z, Y = build_rows([Xs], [Us], dt, fd)
            th = R.eval_library(exps, Z)
            G[a] += th.T @ th
            b[a] += th.T @ Y
            cnt[a] += Xs.shape[0]
    return G, b, cnt


def gram_segments_vectorized(x, u, arm_steps, seq_len, dt, exps, n_arms=4):
    """Vectorised FD-order-1 Gram over all patients (CPU baseline timing and a second form for the
    tests): sample k < L belongs to arm[k] with the forward difference; at every switch and at
    k = L the sample closes the segment of arm[k-1] with the backward difference."""
    N = x.shape[0]
    Lmax = int(seq_len.max())
    K = np.arange(Lmax + 1)[None, :]
    L = np.asarray(seq_len)[:, None]
    fwd = np.zeros((N, Lmax + 1))
    fwd[:, :Lmax] = (x[:, 1:Lmax + 1] - x[:, :Lmax]) / dt
    bwd = np.zeros((N, Lmax + 1))
    bwd[:, 1:] = fwd[:, :Lmax]
    arm_pad = np.full((N, Lmax + 1), -1, dtype=np.int64)
    arm_pad[:, :Lmax] = np.where(K[:, :Lmax] < L, arm_steps[:, :Lmax], -1)
    prev = np.full_like(arm_pad, -1)
    prev[:, 1:] = arm_pad[:, :Lmax]
    close = (prev >= 0) & (arm_pad != prev)
    xs = np.where(K <= L, x[:, :Lmax + 1], 0.0)
    F = exps.shape[0]
    G = np.zeros((n_arms, F, F))
    b = np.zeros((n_arms, F))
    mono = np.ones((N, F))
    for j in range(F):
        for i in range(1, exps.shape[1]):
            mono[:, j] *= u[:, i - 1] ** exps[j, i]
    ex = exps[:, 0]
    for a in range(n_arms):
        m1 = (arm_pad == a).astype(np.float64)
        m2 = (close & (prev == a)).astype(np.float64)
        M = np.stack([(m1 + m2).sum(1), (xs * (m1 + m2)).sum(1), (xs * xs * (m1 + m2)).sum(1),
                      (fwd * m1 + bwd * m2).sum(1), (xs * (fwd * m1 + bwd * m2)).sum(1)], axis=1)
        for i in range(F):
            for j in range(F):
                G[a, i, j] = (mono[:, i] * mono[:, j] * M[:, ex[i] + ex[j]]).sum()
            b[a, i] = (mono[:, i] * M[:, 3 + ex[i]]).sum()
    return G, b


# --------------------------------------------------------------------------------------
# A6 for four arms (sindy.py:289-296)
# --------------------------------------------------------------------------------------
def global_equation_string(coefs, names):
    return " | ".join(f"Treatment {a}: x_dot = {R.equation_terms(c, names)}" for a, c in enumerate(coefs))


# --------------------------------------------------------------------------------------
# Build-defined synthetic 4-arm cohort (layout of the cancer_sim / EQ_5 datasets)
# --------------------------------------------------------------------------------------
# planted per-arm model over [1, x0, u0, x0 u0] (one static, the cancer_sim library):
# arm 0 (no treatment) growth, arms 1..3 (chemo, radio, both) kill terms.
TRUE_COEF_U1 = np.array([
    [0.0, 0.20, 0.0, 0.0],
    [0.0, 0.0, 0.0, -0.60],
    [0.0, -0.30, 0.0, 0.0],
    [0.0, -0.25, 0.0, -0.90],
])


def synthetic_cohort(n, T, rng, switch_p=0.1, noise=0.0, dt=0.1, coef=TRUE_COEF_U1, n_statics=1, min_len=None):
    """x[n, T+1] (Euler-5 of the planted model under per-step arms), u[n, U] ~ N(0.5, 0.05),
    arm_steps[n, T] int64 (Markov: switch to a uniformly drawn other arm with probability switch_p
    per step), seq_len[n] in [min_len, T] (all T when min_len is None)."""
    A = coef.shape[0]
    exps = R.poly_library(1 + n_statics, 2, True)
    u = rng.normal(0.5, 0.05, size=(n, n_statics))
    y = rng.uniform(1.0, 5.0, size=n)
    arms = np.empty((n, T), dtype=np.int64)
    arms[:, 0] = rng.integers(0, A, size=n)
    for k in range(1, T):
        sw = rng.random(n) < switch_p
        other = (arms[:, k - 1] + rng.integers(1, A, size=n)) % A if A > 1 else arms[:, k - 1]
        arms[:, k] = np.where(sw, other, arms[:, k - 1])
    x = np.empty((n, T + 1))
    x[:, 0] = y
    h = dt / R.STEPS_FOR_DT
    mono = np.ones((n, exps.shape[0]))
    for j in range(exps.shape[0]):
        for i in range(1, exps.shape[1]):
            mono[:, j] *= u[:, i - 1] ** exps[j, i]
    ex = exps[:, 0]
    for k in range(T):
        c = coef[arms[:, k]]
        alpha = (c * mono * (ex == 0)).sum(1)
        beta = (c * mono * (ex == 1)).sum(1)
        for _ in range(R.STEPS_FOR_DT):
            y = y + h * (alpha + beta * y)
        x[:, k + 1] = y
    if noise:
        x = x + noise * rng.standard_normal(x.shape)
    if min_len is None:
        seq_len = np.full(n, T, dtype=np.int64)
    else:
        seq_len = rng.integers(min_len, T + 1, size=n).astype(np.int64)
    return x, u, arms, seq_len
