"""GPU parity of the adaptive RK45 rollout on irregular grids (configuration C5) vs oracle/rk45_ref.py
(itself pinned to scipy's solve_ivp in test_rk45_oracle.py).  Tolerance: the same step-size controller
in the same fp64 arithmetic — relative 1e-9 per sample (ulp-level differences can flip an accept/reject
decision near err = 1, which moves the result by at most the RK45 tolerance) and fp64 RMSE <= 1e-6."""
import numpy as np
import pytest
import torch
from scipy.integrate import solve_ivp

from oracle import insite_ref as R
from oracle import rk45_ref as K

pytestmark = pytest.mark.gpu


def _setup(N, seed, per_patient=False):
    rng = np.random.default_rng(seed)
    ex = R.poly_library(3, 2, True)
    t, n = K.irregular_grid(N, rng)
    u = rng.normal(0.5, 0.05, (N, 2))
    arm = (rng.random((N, 60)) < 0.5).astype(np.int8)
    y0 = rng.uniform(1, 50, N)
    coef = np.zeros((2, 7))
    coef[0, 4] = -1.11
    coef[1, 1] = -0.146
    coef[1, 5] = -1.02
    if per_patient:
        coef = np.repeat(coef[None], N, axis=0) * rng.uniform(0.8, 1.2, (N, 1, 1))
    return ex, t, n, u, arm, y0, coef


def _run(dev, ex, t, n, u, arm, y0, coef, order=True, layout="time"):
    """Both layouts: time-major t/y/arm bits [T, N] or patient-major [N, T] (arm bits [N, words])."""
    from insite_amd import ops
    from insite_amd.library import polynomial_library
    lib = polynomial_library(2, 2, True)
    assert np.array_equal(lib.exps.astype(np.int64), ex)
    N, Tm = t.shape
    tn = np.nan_to_num(t, nan=0.0)
    if layout == "patient":
        tt = torch.tensor(np.ascontiguousarray(tn), device=dev)
        bits = ops.pack_arm_bits(torch.tensor(np.ascontiguousarray(arm[:, :Tm]), device=dev), Tm)
    else:
        tt = torch.tensor(np.ascontiguousarray(tn.T), device=dev)
        bits = ops.pack_arm_bits(torch.tensor(np.ascontiguousarray(arm[:, :Tm].T), device=dev), N)
    y, steps = ops.rollout_rk45(torch.tensor(y0, device=dev), torch.tensor(u, device=dev), bits, tt,
                                torch.tensor(n, device=dev), torch.tensor(np.ascontiguousarray(coef), device=dev), lib,
                                order=order, layout=layout)
    torch.cuda.synchronize()
    y = y.cpu().numpy()
    return (y if layout == "patient" else y.T), steps.cpu().numpy()


@pytest.mark.parametrize("layout", ["time", "patient"])
@pytest.mark.parametrize("N,seed", [(1, 0), (63, 1), (200, 2), (257, 3)])
def test_rk45_rollout_matches_oracle(dev, N, seed, layout):
    ex, t, n, u, arm, y0, coef = _setup(N, seed)
    y, steps = _run(dev, ex, t, n, u, arm, y0, coef, layout=layout)
    ref, ref_steps = K.rollout_rk45(y0, u, arm, t, n, coef, ex)
    valid = ~np.isnan(ref)
    assert np.array_equal(np.isnan(y), ~valid)            # rows past each grid untouched (NaN)
    rel = np.abs(y[valid] - ref[valid]) / np.abs(ref[valid])
    assert rel.max() < 1e-9, rel.max()
    assert np.sqrt(np.mean((y[valid] - ref[valid]) ** 2)) <= 1e-6
    assert np.mean(steps == ref_steps) >= 0.99


def test_rk45_rollout_per_patient_coefficients(dev):
    ex, t, n, u, arm, y0, coef = _setup(150, 9, per_patient=True)
    y, _ = _run(dev, ex, t, n, u, arm, y0, coef, layout="patient")
    ref, _ = K.rollout_rk45(y0, u, arm, t, n, coef[0], ex) if False else (None, None)
    # per-patient oracle: each patient with its own [A, F] rows
    for p in range(0, 150, 7):
        rp, _ = K.rollout_rk45(y0[p:p + 1], u[p:p + 1], arm[p:p + 1], t[p:p + 1], n[p:p + 1], coef[p], ex)
        m = ~np.isnan(rp[0])
        assert np.allclose(y[p, m], rp[0, m], rtol=1e-9, atol=0)


def test_rk45_rollout_against_solve_ivp(dev):
    """End-to-end against scipy itself on a few patients (the sub-oracle)."""
    ex, t, n, u, arm, y0, coef = _setup(8, 5)
    y, _ = _run(dev, ex, t, n, u, arm, y0, coef)
    for p in range(8):
        al, be = K.patient_rates(u[p], coef, ex)
        v = y0[p]
        for k in range(n[p] - 1):
            a = arm[p, k]
            if t[p, k + 1] > t[p, k]:
                s = solve_ivp(lambda tt, w: al[a] + be[a] * w, (t[p, k], t[p, k + 1]), [v], method="RK45",
                              rtol=K.RTOL, atol=K.ATOL)
                v = s.y[0, -1]
            assert abs(y[p, k] - v) <= 1e-9 * abs(v)


def test_device_irregular_grid(dev):
    from insite_amd import cohort
    t, n = cohort.irregular_grid(10_000, seed=4, device=dev)
    tc, nc = t.cpu().numpy(), n.cpu().numpy()
    assert nc.min() >= 20 and nc.max() <= 60
    for p in range(0, 10_000, 97):
        g = tc[: nc[p], p]
        assert g[0] == 0.0 and np.all(np.diff(g) >= 0) and g[-1] <= 10.0
        assert np.isnan(tc[nc[p]:, p]).all()


def test_rk45_order_is_a_binned_permutation(dev):
    from insite_amd import ops
    rng = np.random.default_rng(11)
    for N, Tm in [(1, 60), (5000, 60), (70_001, 60), (3000, 2000), (1_000_003, 60)]:
        n = rng.integers(-2, Tm + 5, N).astype(np.int32)
        o = ops.rk45_order(torch.tensor(n, device=dev), Tm).cpu().numpy()
        assert np.array_equal(np.sort(o), np.arange(N))
        key = np.clip(n, 0, min(Tm, 1023))[o]
        assert np.all(np.diff(key) <= 0)                    # descending n_obs (longest rows first)


def test_rk45_row_order_and_layout_do_not_change_outputs(dev):
    """Lane placement and memory layout are scheduling only: binned, random and identity orders in both
    layouts give bit-identical results."""
    ex, t, n, u, arm, y0, coef = _setup(3000, 21)
    y_id, s_id = _run(dev, ex, t, n, u, arm, y0, coef, order=None)
    perm = torch.tensor(np.random.default_rng(3).permutation(3000).astype(np.int32), device=dev)
    runs = [_run(dev, ex, t, n, u, arm, y0, coef, order=o, layout=lay)
            for lay in ("time", "patient") for o in (True, perm, None)]
    for y, s in runs:
        assert np.array_equal(np.isnan(y), np.isnan(y_id))
        assert np.array_equal(y[~np.isnan(y)], y_id[~np.isnan(y_id)]) and np.array_equal(s, s_id)


@pytest.mark.parametrize("layout", ["time", "patient"])
def test_rk45_zero_length_intervals_and_short_grids(dev, layout):
    """Repeated and reversed observation times (y carried over, no attempt), grids of 0/1 observations
    (nothing written), and T_max > 64 (arms read per interval instead of the 64-bit lane mask)."""
    rng = np.random.default_rng(5)
    N, Tm = 300, 90
    ex = R.poly_library(3, 2, True)
    n = rng.integers(0, Tm + 1, N).astype(np.int32)
    n[:3] = [0, 1, 2]
    t = np.full((N, Tm), np.nan)
    for p in range(N):
        g = np.sort(rng.uniform(0.0, 10.0, Tm))
        g[0] = 0.0
        dup = rng.random(Tm) < 0.15
        for k in range(1, Tm):
            if dup[k]:
                g[k] = g[k - 1]                              # zero-length interval
        if p % 7 == 0 and n[p] > 4:
            g[3] = g[2] - 0.5                                # one reversed interval
        t[p, :n[p]] = g[:n[p]]
    u = rng.normal(0.5, 0.05, (N, 2))
    arm = (rng.random((N, Tm)) < 0.5).astype(np.int8)
    y0 = rng.uniform(1, 50, N)
    coef = np.zeros((2, 7))
    coef[0, 4], coef[1, 1], coef[1, 5] = -1.11, -0.146, -1.02
    y, steps = _run(dev, ex, t, n, u, arm, y0, coef, layout=layout)
    ref = np.full((N, Tm), np.nan)
    ref_steps = np.zeros(N, dtype=np.int64)
    for p in range(N):
        al, be = K.patient_rates(u[p], coef, ex)
        v = float(y0[p])
        for k in range(int(n[p]) - 1):
            a = int(arm[p, k])
            if t[p, k + 1] > t[p, k]:
                v, c = K.rk45_interval(lambda w, a=a: al[a] + be[a] * w, v, t[p, k], t[p, k + 1])
                ref_steps[p] += c
            ref[p, k] = v
    valid = ~np.isnan(ref)
    assert np.array_equal(np.isnan(y), ~valid)
    rel = np.abs(y[valid] - ref[valid]) / np.abs(ref[valid])
    assert rel.max() < 1e-9, rel.max()
    assert np.mean(steps == ref_steps) >= 0.99


@pytest.mark.parametrize("layout", ["time", "patient"])
def test_rk45_plan_equals_eager(dev, layout):
    """plan_rollout_rk45 (the C5 bench's per-step call: the counting sort into the plan's own order buffer, then the
    rollout; two C calls) gives bit-identical outputs to rollout_rk45, called twice (the plan reused)."""
    from insite_amd import ops
    from insite_amd.library import polynomial_library
    ex, t, n, u, arm, y0, coef = _setup(2000, 31)
    lib = polynomial_library(2, 2, True)
    N, Tm = t.shape
    tn = np.nan_to_num(t, nan=0.0)
    if layout == "patient":
        tt = torch.tensor(np.ascontiguousarray(tn), device=dev)
        bits = ops.pack_arm_bits(torch.tensor(np.ascontiguousarray(arm[:, :Tm]), device=dev), Tm)
    else:
        tt = torch.tensor(np.ascontiguousarray(tn.T), device=dev)
        bits = ops.pack_arm_bits(torch.tensor(np.ascontiguousarray(arm[:, :Tm].T), device=dev), N)
    args = (torch.tensor(y0, device=dev), torch.tensor(u, device=dev), bits, tt, torch.tensor(n, device=dev),
            torch.tensor(np.ascontiguousarray(coef), device=dev), lib)
    y_e, s_e = ops.rollout_rk45(*args, layout=layout)
    plan = ops.plan_rollout_rk45(*args, layout=layout)
    for _ in range(2):
        y_p, s_p = plan()
        torch.cuda.synchronize()
        assert torch.equal(torch.isnan(y_p), torch.isnan(y_e))
        assert torch.equal(torch.nan_to_num(y_p), torch.nan_to_num(y_e)) and torch.equal(s_p, s_e)


@pytest.mark.parametrize("layout", ["time", "patient"])
def test_rk45_plan_binned_by_attempts_equals_eager(dev, layout):
    """order="attempts" (VERDICT r05 item 7): the plan bins its lanes by the attempt counts the previous call left in
    ``steps`` (the first call: zeros).  Scheduling only -- three consecutive calls give outputs and attempt counts
    bit-identical to the eager n_obs-binned rollout, and the order a call bins by is a permutation sorted by those
    counts (descending)."""
    from insite_amd import ops
    from insite_amd.library import polynomial_library
    ex, t, n, u, arm, y0, coef = _setup(3000, 37)
    lib = polynomial_library(2, 2, True)
    N, Tm = t.shape
    tn = np.nan_to_num(t, nan=0.0)
    if layout == "patient":
        tt = torch.tensor(np.ascontiguousarray(tn), device=dev)
        bits = ops.pack_arm_bits(torch.tensor(np.ascontiguousarray(arm[:, :Tm]), device=dev), Tm)
    else:
        tt = torch.tensor(np.ascontiguousarray(tn.T), device=dev)
        bits = ops.pack_arm_bits(torch.tensor(np.ascontiguousarray(arm[:, :Tm].T), device=dev), N)
    args = (torch.tensor(y0, device=dev), torch.tensor(u, device=dev), bits, tt, torch.tensor(n, device=dev),
            torch.tensor(np.ascontiguousarray(coef), device=dev), lib)
    y_e, s_e = ops.rollout_rk45(*args, layout=layout)
    steps = torch.zeros((N,), dtype=torch.int32, device=dev)
    plan = ops.plan_rollout_rk45(*args, layout=layout, steps=steps, order="attempts")
    for _ in range(3):
        y_p, s_p = plan()
        torch.cuda.synchronize()
        assert torch.equal(torch.isnan(y_p), torch.isnan(y_e))
        assert torch.equal(torch.nan_to_num(y_p), torch.nan_to_num(y_e)) and torch.equal(s_p, s_e)
    o = ops.rk45_order(steps, ops.RK45_ATTEMPT_BINS - 1).cpu().numpy()
    assert np.array_equal(np.sort(o), np.arange(N))
    key = np.clip(steps.cpu().numpy(), 0, ops.RK45_ATTEMPT_BINS - 1)[o]
    assert np.all(np.diff(key) <= 0)
