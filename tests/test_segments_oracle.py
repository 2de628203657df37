"""CPU pins of oracle/segments_ref.py (cancer_sim / EQ_5 discovery).

* the index-form segment walk == a literal transcription of the reference loop
  (libs_m/ct/src/data/pkpd/utils.py:433-462) on one-hot treatments, incl. ragged lengths, switches
  at the first / last step, single-arm patients and seq_len 0 / 1;
* savgol(window 2, polyorder 1) == scipy.signal.savgol_filter itself;
* FD order 1 == forward differences, backward at the last sample (insite_ref.fd_order1, pinned
  in tests/test_oracle.py against the golden fixtures);
* the Gram form (and its vectorised variant) == the row form;
* the planted 4-arm system is recovered from noise-free data.
"""
import numpy as np
import pytest
from scipy.signal import savgol_filter

from oracle import insite_ref as R
from oracle import segments_ref as S


def test_segment_walk_matches_literal_reference_loop():
    rng = np.random.default_rng(0)
    cases = 0
    for _ in range(400):
        T = int(rng.integers(1, 14))
        L = int(rng.integers(0, T + 1))
        A = int(rng.integers(1, 5))
        arm = rng.integers(0, A, size=T)
        if rng.random() < 0.2:
            arm[:] = arm[0]
        onehot = np.eye(4)[arm]
        c = rng.normal(size=T + 1)
        st = rng.normal(size=(T + 1, 2))
        ta, oa, sa = S.split_segments_onehot(onehot, c, st, L)
        b = S.segment_bounds(arm, L)
        assert len(b) == len(oa)
        for (a, s, e), tt, oo, ss in zip(b, ta, oa, sa):
            assert np.argmax(tt.mean(0)) == a                 # utils.py:624
            assert e - s + 1 >= 2
            np.testing.assert_array_equal(oo[:, 0], c[s:e + 1])
            np.testing.assert_array_equal(ss, st[s:e + 1])
            cases += 1
    assert cases > 500


def test_segment_walk_edge_cases():
    assert S.segment_bounds(np.array([2, 2, 2]), 0) == []
    assert S.segment_bounds(np.array([1, 0]), 1) == [(1, 0, 1)]
    assert S.segment_bounds(np.array([0, 1, 1, 3]), 4) == [(0, 0, 1), (1, 1, 3), (3, 3, 4)]
    # a switch at the last observed step still yields a 2-sample final segment
    assert S.segment_bounds(np.array([0, 0, 2, 9]), 3) == [(0, 0, 2), (2, 2, 3)]


@pytest.mark.parametrize("m", [2, 3, 4, 5, 9, 31])
def test_savgol_2_1_matches_scipy(m):
    rng = np.random.default_rng(m)
    x = rng.normal(size=m) * 10
    np.testing.assert_allclose(S.savgol_2_1(x), savgol_filter(x, 2, 1), rtol=0, atol=1e-13)


def test_fd_order1_stencils():
    x = np.array([1.0, 4.0, 9.0, 16.0])
    np.testing.assert_allclose(R.fd_order1(x, 0.5), [6.0, 10.0, 14.0, 14.0])
    np.testing.assert_allclose(R.fd_order1(np.array([2.0, 5.0]), 1.0), [3.0, 3.0])


@pytest.mark.parametrize("n_statics", [1, 2])
def test_gram_forms_agree(n_statics):
    rng = np.random.default_rng(1 + n_statics)
    coef = S.TRUE_COEF_U1 if n_statics == 1 else rng.normal(0, 0.1, size=(4, 7))
    x, u, arm, sl = S.synthetic_cohort(257, 25, rng, switch_p=0.25, noise=0.01, coef=coef, n_statics=n_statics,
                                       min_len=0)
    exps = R.poly_library(1 + n_statics, 2, True)
    G, b, cnt = S.gram_segments(x, u, arm, sl, 0.1, exps)
    G2, b2 = S.gram_segments_vectorized(x, u, arm, sl, 0.1, exps)
    np.testing.assert_allclose(G2, G, rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(b2, b, rtol=1e-12, atol=1e-9)
    np.testing.assert_array_equal(G[:, 0, 0], cnt)
    # the row form: Theta^T Theta of the concatenated per-arm rows
    X, Ul = S.de_segments(x, u, arm, sl)
    for a in range(4):
        Z, Y = S.build_rows(X[a], Ul[a], 0.1)
        th = R.eval_library(exps, Z)
        np.testing.assert_allclose(th.T @ th, G[a], rtol=1e-12, atol=1e-9)
        np.testing.assert_allclose(th.T @ Y, b[a], rtol=1e-12, atol=1e-9)


def test_gram_form_stlsq_equals_row_form():
    rng = np.random.default_rng(7)
    x, u, arm, sl = S.synthetic_cohort(400, 40, rng, switch_p=0.1, noise=0.005, dt=0.05)
    exps = R.poly_library(2, 2, True)
    c_row, ind_row, it_row, _ = S.sindy_fit_segments(x, u, arm, sl, 0.05, threshold=1e-3)
    G, b, _ = S.gram_segments(x, u, arm, sl, 0.05, exps)
    for a in range(4):
        c, ind, it = R.stlsq_gram(G[a], b[a], 1e-3, 0.5)
        assert np.array_equal(ind, ind_row[a]) and it == it_row[a]
        np.testing.assert_allclose(c, c_row[a], rtol=1e-8, atol=1e-10)


def test_planted_four_arm_system_recovered():
    rng = np.random.default_rng(3)
    x, u, arm, sl = S.synthetic_cohort(600, 200, rng, switch_p=0.05, dt=0.01)
    coef, ind, _, _ = S.sindy_fit_segments(x, u, arm, sl, 0.01, threshold=0.1)
    np.testing.assert_array_equal(ind, S.TRUE_COEF_U1 != 0)
    assert np.max(np.abs(coef - S.TRUE_COEF_U1)) < 0.02


def test_empty_arm_raises_like_pysindy():
    rng = np.random.default_rng(4)
    x, u, arm, sl = S.synthetic_cohort(20, 10, rng, switch_p=0.0)
    arm[:] = 1
    with pytest.raises(ValueError, match="no treatment segments"):
        S.sindy_fit_segments(x, u, arm, sl, 0.1)


def test_equation_string_has_four_treatments():
    names = ["1", "x0", "u0", "x0 u0"]
    s = S.global_equation_string(S.TRUE_COEF_U1, names)
    assert s.count("Treatment ") == 4 and "Treatment 3: x_dot = +-0.25*x0+-0.9*x0*u0" in s
