"""CPU: host logic of the ablation models (no GPU): the joint model's fold into per-combination arms
(SINDY._fold_joint) evaluates the same RHS as the joint library, the degree-4 / joint library tables
follow pysindy's column order, and the oracle's Gram form equals its row form on both ablations."""
import numpy as np
import pytest

from oracle import insite_ref as R


def test_joint_library_and_fold_equal_joint_rhs():
    from insite_amd.library import polynomial_library
    from insite_amd.sindy import SINDY
    lib = polynomial_library(2, 2, True, n_inputs=1)
    assert lib.get_feature_names() == ["1", "x0", "u0", "u1", "u2", "x0 u0", "x0 u1", "x0 u2", "u0 u1", "u0 u2", "u1 u2"]
    m = SINDY.__new__(SINDY)
    m.library = lib
    rng = np.random.default_rng(0)
    c = rng.normal(size=(1, lib.n_terms))
    red, folded = m._fold_joint(c)
    y, stat = rng.uniform(1, 50, 64), rng.normal(0.5, 0.05, (64, 2))
    for a in (0, 1):
        u_joint = np.concatenate([np.full((64, 1), float(a)), stat], axis=1)
        want = R.rhs_literal(y, u_joint, np.repeat(c, 64, 0), lib.exps.astype(np.int64))
        got = R.rhs_literal(y, stat, np.repeat(folded[a][None], 64, 0), red.exps.astype(np.int64))
        np.testing.assert_allclose(got, want, rtol=1e-12)


def test_two_input_fold():
    from insite_amd.library import polynomial_library
    from insite_amd.sindy import SINDY
    lib = polynomial_library(1, 2, True, n_inputs=2)          # cancer_sim joint: (x0, chemo, radio, static)
    m = SINDY.__new__(SINDY)
    m.library = lib
    c = np.random.default_rng(1).normal(size=(1, lib.n_terms))
    red, folded = m._fold_joint(c)
    assert folded.shape[0] == 4
    y, stat = np.linspace(1, 40, 16), np.linspace(-1, 1, 16)[:, None]
    for code in range(4):
        bits = np.array([code & 1, code >> 1], dtype=np.float64)
        u_joint = np.concatenate([np.repeat(bits[None], 16, 0), stat], axis=1)
        want = R.rhs_literal(y, u_joint, np.repeat(c, 16, 0), lib.exps.astype(np.int64))
        got = R.rhs_literal(y, stat, np.repeat(folded[code][None], 16, 0), red.exps.astype(np.int64))
        np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-12)


def test_degree4_library_order_matches_pysindy_layout():
    from insite_amd.library import polynomial_library
    lib = polynomial_library(2, 4, False)
    np.testing.assert_array_equal(lib.exps, R.poly_library(3, 4, False))
    names = lib.get_feature_names()
    assert len(names) == 35 and names[:4] == ["1", "x0", "u0", "u1"] and names[4] == "x0^2" and names[-1] == "u1^4"


@pytest.mark.parametrize("degree,inter", [(4, False), (2, True)])
def test_oracle_gram_form_equals_row_form(degree, inter):
    coll = R.make_collection("EQ_4_A", {"train": 60, "val": 4, "test": 4}, seed=3, with_tests=False)
    tr = coll["train"]
    x, u, arm, rows = R.de_format(tr.data, tr.scaling_params)
    exps = R.poly_library(3, degree, inter)
    G, b = R.gram_moments(x, u, arm, rows, 1 / 6, exps)
    X, U = R.de_lists(x, u, arm, rows)
    for a in range(2):
        Z, Y = R.build_regression(X[a], U[a], 1 / 6)
        th = R.eval_library(exps, Z)
        np.testing.assert_allclose(G[a], th.T @ th, rtol=1e-12)
        np.testing.assert_allclose(b[a], th.T @ Y, rtol=1e-12, atol=1e-9)
