"""CPU tests of the multi-state restatement (oracle/multistate_ref.py, configuration C3) and of the
host side of its ABI.  C3 has no reference counterpart: the restatement is pinned by the reference's
own one-state semantics it reuses (insite_ref, itself pinned in test_oracle.py), by recovering the
planted truth model, and by the identities below."""
import ctypes

import numpy as np
import pytest

from oracle import insite_ref as R
from oracle import multistate_ref as M


def test_library_is_pysindy_order_over_states_then_input():
    ex = M.c3_library()
    assert ex.shape == (22, 6)
    from insite_amd.multistate import ms_library
    assert np.array_equal(ms_library(5, 1, True).exps.astype(np.int64), ex)
    names = R.library_names(ex, M.INPUT_NAMES_C3)
    assert names[:7] == ["1", "x1", "x2", "x3", "x4", "x5", "a"] and names[7] == "x1 x2" and names[-1] == "x5 a"


def test_truth_rollout_reproduces_the_cohort():
    """The cohort is the RK4-10 integration of the truth; the S-state rollout with the same
    integrator and the truth coefficients reproduces it (up to the fp32 storage)."""
    x, a = M.c3_cohort(64, 80, seed=5)
    ex = M.c3_library()
    y = M.ms_rollout(x[:, 0].astype(np.float64), a, M.c3_truth_coef(ex), ex, M.DT_C3, "rk4", substeps=10, drop=0.0)
    assert np.allclose(y[:, :-1], x[:, 1:], rtol=1e-6, atol=1e-6)


def test_gram_loop_equals_vectorised():
    x, a = M.c3_cohort(40, 120, seed=3)
    ex = M.c3_library()
    G, B = M.ms_gram(x, a, np.full(40, 120), M.DT_C3, ex)
    G2, B2 = M.ms_gram_vectorized(x, a, M.DT_C3, ex)
    assert np.allclose(G, G2, rtol=1e-12, atol=1e-9) and np.allclose(B, B2, rtol=1e-12, atol=1e-9)


def test_gram_rows_ragged_and_short_are_per_trajectory():
    """Ragged rows: each patient is its own trajectory (multiple_trajectories=True); < 5 rows are
    skipped (pysindy would raise)."""
    x, a = M.c3_cohort(6, 30, seed=4)
    ex = M.c3_library()
    rows = np.array([30, 4, 5, 7, 9, 12])
    G, B = M.ms_gram(x, a, rows, M.DT_C3, ex)
    G2 = np.zeros_like(G)
    B2 = np.zeros_like(B)
    for i, L in enumerate(rows):
        if L < 5:
            continue
        Z, Y = M.ms_regression(x[i], a[i], L, M.DT_C3)
        th = R.eval_library(ex, Z)
        G2 += th.T @ th
        B2 += th.T @ Y
    assert np.allclose(G, G2) and np.allclose(B, B2)


def test_discovery_recovers_the_planted_c3_system():
    coef, mask, truth = M.ms_pipeline(N=200, T=400)
    assert np.array_equal(mask, truth != 0)
    # chain / tumour equations are exact up to the FD error; the dosed x1 equation is biased by the
    # derivative smear at treatment switches (documented in DESIGN.md)
    assert np.abs(coef[1:] - truth[1:]).max() < 2e-3
    assert np.abs(coef[0] - truth[0]).max() < 0.1


def test_stlsq_per_target_matches_row_form():
    """ms_stlsq (normal equations) == insite_ref.stlsq on the materialised rows, per target."""
    x, a = M.c3_cohort(60, 150, seed=8)
    ex = M.c3_library()
    G, B = M.ms_gram_vectorized(x, a, M.DT_C3, ex)
    coef, mask, _ = M.ms_stlsq(G, B)
    Zs, Ys = zip(*[M.ms_regression(x[i], a[i], 150, M.DT_C3) for i in range(60)])
    th = R.eval_library(ex, np.concatenate(Zs))
    Y = np.concatenate(Ys)
    for s in range(5):
        c, ind, _ = R.stlsq(th, Y[:, s], M.THRESHOLD_C3, M.ALPHA_C3)
        assert np.array_equal(ind, mask[s])
        assert np.abs(c - coef[s]).max() < 1e-8


def test_ms_abi_rejects_bad_arguments_on_host():
    from insite_amd import _lib
    L = _lib.load()
    ex = np.ascontiguousarray(M.c3_library(), dtype=np.int8)
    exp_p = ex.ctypes.data_as(ctypes.c_void_p)
    vp = ctypes.c_void_p
    # unsupported state count / library, and bad leading dimensions, fail before any launch
    assert L.insite_gram_ms_f32(vp(0), 10, 8, 4, vp(0), 0, vp(0), 10, exp_p, 22, 0, 0.1, vp(8), vp(8), vp(8), 1 << 20,
                                vp(0)) == -2
    assert L.insite_gram_ms_f32(vp(0), 5, 8, 5, vp(0), 0, vp(0), 10, exp_p, 22, 0, 0.1, vp(8), vp(8), vp(8), 1 << 20,
                                vp(0)) == -1
    bad = ex.copy()
    bad[7] = bad[8]
    assert L.insite_rollout_ms_f32(vp(8), 10, vp(8), 1, vp(8), bad.ctypes.data_as(vp), 22, 5, 10, 4, 0.1, 1, 1,
                                   1e-3, vp(8), 10, vp(0)) == -2
    assert L.insite_stlsq_wave_f64(vp(8), vp(8), 40, 5, 0.1, 0.5, 100, 1, vp(8), vp(0), vp(0), vp(0)) == -1
    assert L.insite_gram_ms_workspace_bytes(1_000_000) == 512 * 3 * 256 * 8


def test_ms_ops_refuse_host_tensors():
    import torch
    from insite_amd import multistate as MS
    lib = MS.ms_library()
    with pytest.raises(ValueError):
        MS.gram_ms(torch.zeros((8, 5, 4), dtype=torch.float32), None, lib, 0.1)
