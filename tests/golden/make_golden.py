#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (committed; re-run to refresh).

The reference (Python/JAX + pysindy) cannot be imported in this container (jax, pysindy absent:
ordinary ModuleNotFoundError), so the vectors come from the CPU restatement
``oracle/insite_ref.py`` and are cross-checked HERE, at generation time, against the primitives
pysindy delegates to (scipy.signal.savgol_filter, sklearn ridge_regression, numpy lstsq) and
against the reference's own anchors (in-module known answer y(t)=t, utils.py:759-858; published
log equations, results/2_main_table/final_with_insite.txt:126,182).  Every file is a plain .npz
(no pickled objects: load with numpy's default allow_pickle=False).

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import insite_ref as R  # noqa: E402


def _save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path)} B)")


def stencils():
    from scipy.signal import savgol_filter
    rng = np.random.default_rng(20240601)
    out = {}
    for L in (5, 6, 7, 12, 60):
        x = rng.uniform(1.0, 50.0, size=L)
        dt = 10.0 / 60.0
        sg = savgol_filter(x, 5, 3, mode="interp")
        mine = R.savgol_5_3(x)
        assert np.allclose(mine, sg, rtol=1e-13, atol=1e-12), L
        xs, xd = R.smoothed_fd4(x, dt)
        out[f"x_{L}"] = x
        out[f"savgol_{L}"] = sg
        out[f"smoothed_fd4_{L}"] = xd
        out[f"fd4_{L}"] = R.fd_order4(x, dt)
        out[f"fd1_{L}"] = R.fd_order1(x, dt)
    out["dt"] = np.float64(10.0 / 60.0)
    _save("stencils.npz", **out)


def library():
    out = {}
    for tag, (n_in, deg, io, names) in {
        "u2_d2_io": (3, 2, True, ["x0", "u0", "u1"]),
        "u1_d2_full": (2, 2, False, ["x0", "u0"]),
        "u3_d2_io": (4, 2, True, ["x0", "u0", "u1", "u2"]),
    }.items():
        e = R.poly_library(n_in, deg, io)
        out[f"exps_{tag}"] = e.astype(np.int8)
        out[f"names_{tag}"] = np.array(R.library_names(e, names))
    assert list(out["names_u2_d2_io"]) == ["1", "x0", "u0", "u1", "x0 u0", "x0 u1", "u0 u1"]
    _save("library.npz", **out)


def discovery(eq, n=200, T=60, seed=0):
    from sklearn.linear_model import ridge_regression
    coll = R.make_collection(eq, {"train": n, "val": 4, "test": 4}, seq_length=T, seed=seed, with_tests=False)
    tr = coll["train"]
    x, u, arm, rows = R.de_format(tr.data, tr.scaling_params)
    dt = R.MAX_TIME_HORIZON / T
    exps = R.poly_library(3, 2, True)
    names = R.library_names(exps, ["x0", "u0", "u1"])
    G, b = R.gram_moments(x, u, arm, rows, dt, exps)
    X, U = R.de_lists(x, u, arm, rows)
    coefs, masks, its, margins = [], [], [], []
    for a in range(2):
        Z, Y = R.build_regression(X[a], U[a], dt)
        th = R.eval_library(exps, Z)
        # sub-oracle: the first ridge pass equals sklearn's Cholesky ridge on all columns
        w_sk = ridge_regression(th, Y, alpha=0.5, solver="cholesky")
        assert np.allclose(R.ridge_cholesky(th, Y, 0.5), w_sk, rtol=1e-9, atol=1e-10)
        c, ind, it = R.stlsq(th, Y, 0.1, 0.5)
        cg, indg, itg = R.stlsq_gram(G[a], b[a], 0.1, 0.5)
        assert np.array_equal(ind, indg) and it == itg and np.max(np.abs(c - cg)) < 1e-9
        coefs.append(c)
        masks.append(ind.astype(np.int8))
        its.append(it)
        # distance of the last ridge pass from the threshold (fixtures avoid near-ties)
        S = np.nonzero(ind)[0]
        A_ = G[a][np.ix_(S, S)] + 0.5 * np.eye(S.size)
        margins.append(float(np.min(np.abs(np.linalg.solve(A_, b[a][S]))) - 0.1) if S.size else 0.0)
    joint = np.stack(coefs)
    eqs = R.global_equation_string(joint, names)
    _save(f"discovery_{eq.lower()}.npz", x=x, u=u, arm=arm.astype(np.int8), rows=rows.astype(np.int32),
          dt=np.float64(dt), G=G, b=b, coef=joint, mask=np.stack(masks), iters=np.array(its, np.int32),
          margin=np.array(margins), equation=np.array(eqs), threshold=np.float64(0.1), alpha=np.float64(0.5))
    return joint, eqs


def rollouts():
    rng = np.random.default_rng(77)
    N, T, A = 64, 20, 2
    exps = R.poly_library(3, 2, True)
    F = exps.shape[0]
    y0 = rng.uniform(1, 50, N)
    u = rng.normal(0.5, 0.05, (N, 2))
    arm = rng.integers(0, A, (N, T)).astype(np.int8)
    coef = np.zeros((A, F))
    coef[0, 4] = -1.1104
    coef[1, 1] = -0.1467
    coef[1, 5] = -1.0209
    coef[0, 2] = 5e-4          # below the 1e-3 RHS filter: must be dropped
    per = coef[None] * (1.0 + 0.05 * rng.normal(size=(N, A, F)))
    dt = R.MAX_TIME_HORIZON / T
    out = dict(y0=y0, u=u, arm=arm, coef=coef, coef_per_patient=per, dt=np.float64(dt), exps=exps.astype(np.int8))
    out["euler5"] = R.rollout(y0, u, arm, coef, exps, dt, "euler5")
    out["rk4"] = R.rollout(y0, u, arm, coef, exps, dt, "rk4")
    out["euler3"] = R.rollout(y0, u, arm, coef, exps, dt, "euler", substeps=3)
    out["euler5_per_patient"] = R.rollout(y0, u, arm, per, exps, dt, "euler5")
    # the reference's in-module known answer (utils.py:759-858): dy/dt = 1 -> y(t) = t
    one = np.zeros((A, F))
    one[:, 0] = 1.0
    t = R.rollout(np.zeros(3), np.full((3, 2), 0.5), np.zeros((3, 60), np.int8), one, exps, R.STANDARD_DT, "euler5")
    assert np.mean((t - np.arange(1, 61)[None] * R.STANDARD_DT) ** 2) < 1e-16
    _save("rollout.npz", **out)


def metrics():
    rng = np.random.default_rng(5)
    N, T = 40, 12
    pred = rng.uniform(1, 50, (N, T, 1))
    target = pred + rng.normal(0, 0.5, (N, T, 1))
    sl = rng.integers(2, T + 1, N)
    active = (np.arange(T)[None, :, None] < sl[:, None, None]).astype(np.float64)
    o, a_, l = R.masked_rmse(pred, target, active, one_step_counterfactual=True)
    nst = R.n_step_rmses(pred, target, active)
    _save("metrics.npz", pred=pred, target=target, active=active, rmse_orig=np.float64(o), rmse_all=np.float64(a_),
          rmse_last=np.float64(l), n_step=nst)


if __name__ == "__main__":
    stencils()
    library()
    ja, ea = discovery("EQ_4_A")
    jc, ec = discovery("EQ_4_C")
    print(ea)
    print(ec)
    rollouts()
    metrics()
