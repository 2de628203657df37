"""GPU parity of the multi-state path (configuration C3) through the C ABI vs oracle/multistate_ref.py.

Tolerances: Gram/moments relative 1e-10 (fp64 sums, same fp32 inputs); discovered support identical and
coefficient L-inf < 1e-8 against the restatement's STLSQ on the same Gram; fp32 rollouts against the
fp64 restatement: max relative error 1e-4 (fp32 arithmetic over <= 200 RK4 steps)."""
import numpy as np
import pytest
import torch

from oracle import insite_ref as R
from oracle import multistate_ref as M

pytestmark = pytest.mark.gpu


def _x_dev(x, dev, pad=3):
    """[N, T, S] numpy -> device [T, S, N + pad] float32 (padding NaN: stray reads poison sums)."""
    N, T, S = x.shape
    out = np.full((T, S, N + pad), np.nan, dtype=np.float32)
    out[:, :, :N] = np.transpose(x, (1, 2, 0))
    return torch.tensor(out, device=dev)


def _bits(a, dev):
    from insite_amd.ops import pack_arm_bits
    return pack_arm_bits(torch.tensor(np.ascontiguousarray(a.T), device=dev), a.shape[0])


def _lib(n_inputs=1, inter=True):
    from insite_amd.multistate import ms_library
    return ms_library(5, n_inputs, inter)


@pytest.mark.parametrize("n_inputs,inter", [(1, True), (0, True), (0, False)])
@pytest.mark.parametrize("N,T", [(200, 48), (67, 130), (130, 300)])  # (67, 130) / (130, 300): 2 / 4 time chunks per tile
def test_gram_ms_matches_oracle(dev, n_inputs, inter, N, T):
    from insite_amd import multistate as MS
    x, a = M.c3_cohort(N, T, seed=11)
    rng = np.random.default_rng(1)
    rows = rng.integers(0, T + 1, N).astype(np.int32)
    rows[:10] = [0, 4, 5, 6, 7, 8, 9, 10, T, T - 1]
    lib = _lib(n_inputs, inter)
    ex = lib.exps.astype(np.int64)
    if n_inputs:
        G_ref, B_ref = M.ms_gram(x, a, rows, M.DT_C3, ex)
    else:  # library over the states only: Z without the input column
        F = ex.shape[0]
        G_ref, B_ref = np.zeros((F, F)), np.zeros((F, 5))
        for i in range(N):
            L = int(rows[i])
            if L < 5:
                continue
            Z, Y = M.ms_regression(x[i], a[i], L, M.DT_C3)
            th = R.eval_library(ex, Z[:, :5])
            G_ref += th.T @ th
            B_ref += th.T @ Y
    G, B = MS.gram_ms(_x_dev(x, dev), _bits(a, dev) if n_inputs else None, lib, M.DT_C3,
                      rows=torch.tensor(rows, device=dev), n_patients=N)
    torch.cuda.synchronize()
    assert np.allclose(G.cpu().numpy(), G_ref, rtol=1e-10, atol=1e-8)
    assert np.allclose(B.cpu().numpy(), B_ref, rtol=1e-10, atol=1e-8)


def test_stlsq_wave_matches_oracle_on_c3_gram(dev):
    from insite_amd import multistate as MS
    x, a = M.c3_cohort(300, 300, seed=2)
    ex = M.c3_library()
    G, B = M.ms_gram_vectorized(x, a, M.DT_C3, ex)
    c_ref, m_ref, _ = M.ms_stlsq(G, B)
    coef, mask, iters = MS.stlsq_wave(torch.tensor(G, device=dev), torch.tensor(B, device=dev), M.THRESHOLD_C3,
                                      M.ALPHA_C3)
    torch.cuda.synchronize()
    assert np.array_equal(mask.cpu().numpy() != 0, m_ref)
    assert np.abs(coef.cpu().numpy() - c_ref).max() < 1e-8
    assert (iters.cpu().numpy() > 0).all()


@pytest.mark.parametrize("F", [7, 16, 22, 32])
def test_stlsq_wave_random_systems(dev, F):
    """Random SPD systems with a sparse planted solution: the wave solver == the restatement."""
    from insite_amd import multistate as MS
    rng = np.random.default_rng(F)
    X = rng.normal(size=(400, F))
    S = 6
    C = rng.normal(size=(S, F)) * (rng.random((S, F)) < 0.3)
    Y = X @ C.T + 0.05 * rng.normal(size=(400, S))
    G, B = X.T @ X, X.T @ Y
    coef, mask, _ = MS.stlsq_wave(torch.tensor(G, device=dev), torch.tensor(B, device=dev), 0.2, 0.5)
    torch.cuda.synchronize()
    for s in range(S):
        c, ind, _ = R.stlsq_gram(G, B[:, s], 0.2, 0.5)
        assert np.array_equal(mask.cpu().numpy()[s] != 0, ind)
        assert np.abs(coef.cpu().numpy()[s] - c).max() < 1e-8


def test_stlsq_wave_agrees_with_the_one_thread_solver(dev):
    from insite_amd import multistate as MS
    from insite_amd import ops
    rng = np.random.default_rng(7)
    X = rng.normal(size=(200, 7))
    Y = X @ np.array([[0, 1.5, 0, 0, -2.0, 0, 0.3], [0.7, 0, 0, 0, 0, 0, 0]]).T + 0.01 * rng.normal(size=(200, 2))
    G, B = X.T @ X, X.T @ Y
    c1, m1, _ = MS.stlsq_wave(torch.tensor(G, device=dev), torch.tensor(B, device=dev), 0.1, 0.5)
    Gs = torch.tensor(np.stack([G, G]), device=dev)
    c2, m2, _ = ops.stlsq(Gs, torch.tensor(np.ascontiguousarray(B.T), device=dev), 0.1, 0.5)
    torch.cuda.synchronize()
    assert torch.equal(m1, m2)
    assert (c1 - c2).abs().max().item() < 1e-12


def test_c3_discovery_end_to_end(dev):
    """numpy cohort -> device Gram + STLSQ: the planted support, and the restatement's coefficients."""
    from insite_amd import multistate as MS
    x, a = M.c3_cohort(256, 400, seed=2)
    ex = M.c3_library()
    G_ref, B_ref = M.ms_gram_vectorized(x, a, M.DT_C3, ex)
    c_ref, m_ref, _ = M.ms_stlsq(G_ref, B_ref)
    coef, mask, iters, G, B = MS.fit_ms(_x_dev(x, dev, pad=0), _bits(a, dev), _lib(), M.DT_C3)
    torch.cuda.synchronize()
    truth = M.c3_truth_coef(ex)
    assert np.array_equal(mask.cpu().numpy() != 0, truth != 0)
    assert np.array_equal(mask.cpu().numpy() != 0, m_ref)
    assert np.abs(coef.cpu().numpy() - c_ref).max() < 1e-8


@pytest.mark.parametrize("method,sub", [("rk4", 1), ("rk4", 3), ("euler", 5)])
@pytest.mark.parametrize("N", [1, 100, 333])
def test_rollout_ms_matches_oracle(dev, method, sub, N):
    from insite_amd import multistate as MS
    rng = np.random.default_rng(N)
    ex = M.c3_library()
    coef = M.c3_truth_coef(ex) * (1 + 0.1 * rng.normal(size=(5, 22)) * (M.c3_truth_coef(ex) != 0))
    coef[2, 9] = 0.02          # a small extra term: inside the RHS (> drop)
    coef[3, 12] = 5e-4         # below the 1e-3 drop: excluded (utils.py:388)
    T = 150
    a = M.treatment_markov(N, T, rng, 0.3, 0.05)
    y0 = np.stack([rng.uniform(0, 1, N) for _ in range(4)] + [rng.uniform(1, 5, N)], axis=0).astype(np.float32)
    ref = M.ms_rollout(y0.T.astype(np.float64), a, coef, ex, M.DT_C3, method, substeps=sub)
    y = MS.rollout_ms(torch.tensor(y0, device=dev), _bits(a, dev), torch.tensor(coef, device=dev), _lib(), M.DT_C3,
                      T, method=method, substeps=sub)
    torch.cuda.synchronize()
    got = np.transpose(y.cpu().numpy(), (2, 0, 1))  # [N, T, S]
    rel = np.abs(got - ref) / np.maximum(np.abs(ref), 1e-2)
    assert rel.max() < 1e-4, rel.max()


def test_rollout_ms_padding_untouched(dev):
    from insite_amd import multistate as MS
    N, T = 70, 40
    out = torch.full((T, 5, N + 9), 7.0, dtype=torch.float32, device=dev)
    y0 = torch.rand((5, N), device=dev)
    a = torch.zeros((T, 3), dtype=torch.int32, device=dev)
    coef = torch.tensor(M.c3_truth_coef(M.c3_library()), device=dev)
    y_full = MS.rollout_ms(y0, a, coef, _lib(), M.DT_C3, T)
    ld = N + 9
    # write through a [T, S, ld] buffer: the columns past N stay untouched
    from insite_amd import _lib as L_
    import ctypes
    L = L_.load()
    tab = _lib().table()
    st = L.insite_rollout_ms_f32(ctypes.c_void_p(y0.data_ptr()), N, ctypes.c_void_p(a.data_ptr()), 3,
                                 ctypes.c_void_p(coef.data_ptr()), tab.ctypes.data_as(ctypes.c_void_p), 22, 5, N, T,
                                 M.DT_C3, 1, 1, 1e-3, ctypes.c_void_p(out.data_ptr()), ld, ctypes.c_void_p(0))
    assert st == 0
    torch.cuda.synchronize()
    assert (out[:, :, N:] == 7.0).all()
    assert torch.equal(out[:, :, :N], y_full)


def test_synthetic_c3_device_cohort_recovers_truth(dev):
    from insite_amd import multistate as MS
    coh = MS.synthetic_c3(4096, 500, seed=2, device=dev)
    assert bool(torch.isfinite(coh.x).all())
    coef, mask, iters, G, B = MS.fit_ms(coh.x, coh.a, coh.lib, coh.dt)
    torch.cuda.synchronize()
    truth = MS.c3_truth_coef(coh.lib, device=dev)
    assert torch.equal(mask != 0, truth != 0)
    assert (coef[1:] - truth[1:]).abs().max().item() < 5e-3


@pytest.mark.parametrize("method,sub", [("rk4", 1), ("euler", 2)])
@pytest.mark.parametrize("inputs", [True, False])
def test_sparse_rollout_equals_dense(dev, method, sub, inputs):
    """insite_rollout_ms_sparse_f32 (support-specialised kernel generated with hipRTC) evaluates only the
    model's terms in the library's column order: bitwise the dense kernel's trajectories; an extra small
    term above the drop threshold outside the given support makes the launch take the dense RHS (still
    equal); a term below the threshold is dropped either way."""
    from insite_amd import multistate as MS
    rng = np.random.default_rng(7)
    ex = M.c3_library()
    truth = M.c3_truth_coef(ex)
    coef = truth * (1 + 0.1 * rng.normal(size=truth.shape) * (truth != 0))
    coef[3, 12] = 5e-4                       # below drop: not in the model
    N, T = 3000, 97
    a = M.treatment_markov(N, T, rng, 0.3, 0.05)
    bits = _bits(a, dev) if inputs else None
    lib = _lib() if inputs else _lib(n_inputs=0)
    if not inputs:                           # a sparse model over the 16 state-only columns
        coef = np.zeros((5, lib.n_terms))
        for s_ in range(5):
            coef[s_, 1 + s_] = -0.5
        coef[1, 1], coef[4, 10], coef[2, 0] = 0.4, -0.2, 0.05
    y0 = torch.tensor(np.stack([rng.uniform(0, 1, N) for _ in range(4)] + [rng.uniform(1, 5, N)]).astype(np.float32),
                      device=dev)
    c = torch.tensor(coef, device=dev)
    support = np.abs(coef) > 1e-3
    y_dense = MS.rollout_ms(y0, bits, c, lib, M.DT_C3, T, method=method, substeps=sub)
    y_sparse = MS.rollout_ms(y0, bits, c, lib, M.DT_C3, T, method=method, substeps=sub, support=support)
    torch.cuda.synchronize()
    assert torch.equal(y_sparse, y_dense)
    # a stale support (one model term missing): the launch falls back to the dense RHS
    stale = support.copy()
    stale[np.argwhere(support)[0][0], np.argwhere(support)[0][1]] = False
    y_stale = MS.rollout_ms(y0, bits, c, lib, M.DT_C3, T, method=method, substeps=sub, support=stale)
    torch.cuda.synchronize()
    assert torch.equal(y_stale, y_dense)
