"""GPU: the general one-state path (csrc/insite_gen.hip) against the oracle — the reference's two
library ablations:

* degree-4 library (PolynomialLibrary(degree=4, interaction_only=False), reference sindy.py:185-186,
  run.py:208 ABLATION_MORE_COMPLEX_BASIS_FUNCTIONS): F = 35, state exponents up to 4 — Gram via power
  moments, STLSQ one wavefront per arm (F <= 64), stage-evaluated Euler-5 / RK4 rollout of the polynomial
  RHS;
* joint ("one ODE") model (joint_model + multilabel treatments, run.py:198-201; DE format
  pkpd/utils.py:486-497, 639-672): one regression with the per-step treatment bit(s) as library inputs.

Both on the reference's own EQ_4 cohorts (oracle/ref_cohort.py).  The degree-4 normal equations have
condition numbers ~1e16 (the oracle's row form and Gram form already differ by ~3e-9 on them), so
coefficients are compared at rtol 1e-6 there; everything else at the usual 1e-10 / 1e-8.
"""
import numpy as np
import pytest
import torch

from oracle import insite_ref as R
from oracle import ref_cohort as RC
from oracle import segments_ref as SG

pytestmark = pytest.mark.gpu


def _dl(a, dev, dtype=None):
    return torch.as_tensor(np.ascontiguousarray(a), device=dev, dtype=dtype)


@pytest.fixture(scope="module")
def c_coll():
    return RC.make_collection("EQ_4_C")


@pytest.fixture(scope="module")
def c_coll_ml():
    return RC.make_collection("EQ_4_C", treatment_mode="multilabel")


@pytest.mark.parametrize("layout", ["patient", "time"])
def test_degree4_gram_matches_oracle(dev, c_coll, layout):
    from insite_amd import ops
    from insite_amd.library import polynomial_library
    tr = c_coll["train"]
    x, u, arm, rows = R.de_format(tr.data, tr.scaling_params)
    rows = rows.copy()
    rows[::7] -= 11                                            # ragged rows
    lib = polynomial_library(2, 4, False)
    assert lib.n_terms == 35
    exps = lib.exps.astype(np.int64)
    xt = _dl(x if layout == "patient" else x.T, dev)
    G, b = ops.gen_gram(xt, _dl(u, dev), _dl(rows, dev, torch.int32), R.STANDARD_DT, lib,
                        group=_dl(arm, dev, torch.int8), n_groups=2, layout=layout)
    Gr, br = R.gram_moments(x, u, arm, rows, R.STANDARD_DT, exps)
    G, b = G.cpu().numpy(), b.cpu().numpy()
    for a in range(2):
        np.testing.assert_allclose(G[a], Gr[a], rtol=1e-11, atol=1e-13 * np.abs(Gr[a]).max())
        np.testing.assert_allclose(b[a], br[a], rtol=1e-11, atol=1e-13 * np.abs(br[a]).max())
        np.testing.assert_array_equal(G[a], G[a].T)


def test_degree4_stlsq_and_rollout_match_oracle(dev, c_coll):
    from insite_amd import ops
    from insite_amd.library import polynomial_library
    tr = c_coll["train"]
    x, u, arm, rows = R.de_format(tr.data, tr.scaling_params)
    lib = polynomial_library(2, 4, False)
    coef, mask, iters, G, b = ops.gen_sindy_fit(_dl(x, dev), _dl(u, dev), _dl(rows, dev, torch.int32), R.STANDARD_DT,
                                                lib, 0.1, 0.5, group=_dl(arm, dev, torch.int8), n_groups=2)
    Gh, bh = G.cpu().numpy(), b.cpu().numpy()
    ref = np.stack([R.stlsq_gram(Gh[a], bh[a], 0.1, 0.5)[0] for a in range(2)])
    c = coef.cpu().numpy()
    assert (iters.cpu().numpy() > 0).all()
    assert np.array_equal(mask.cpu().numpy() != 0, ref != 0)
    np.testing.assert_allclose(c, ref, rtol=1e-6, atol=1e-9)
    # stage-evaluated polynomial rollout (both integrators, both layouts) vs the oracle's literal RHS
    one = c_coll["test_cf_one_step"]
    prev, stat = R.unscale_inputs(one.data, one.scaling_params)
    arms = np.argmax(one.data["current_treatments"], axis=-1).astype(np.int8)
    sel = np.arange(0, prev.shape[0], 7)
    rhs = np.where(np.abs(ref) > 1e-3, ref, 0.0)
    for method in ("euler5", "rk4"):
        want = R.rollout(prev[sel, 0], stat[sel], arms[sel], rhs, lib.exps.astype(np.int64), R.STANDARD_DT, method)
        for layout in ("patient", "time"):
            a_ = arms[sel] if layout == "patient" else arms[sel].T
            y = ops.rollout(_dl(prev[sel, 0], dev), _dl(stat[sel], dev), _dl(a_, dev), _dl(rhs, dev), lib, R.STANDARD_DT,
                            method=method, drop_below=0.0, layout=layout)
            got = y.cpu().numpy() if layout == "patient" else y.cpu().numpy().T
            np.testing.assert_allclose(got, want, rtol=1e-11, atol=1e-12)


def test_stlsq_wave64_matches_oracle_on_random_systems(dev):
    """insite_stlsq_f64 dispatches F > 9 to the one-wavefront-per-system solver: random SPD systems
    (F = 11, 22, 35, 64) with planted sparse solutions, several thresholds."""
    from insite_amd import ops
    rng = np.random.default_rng(11)
    for F in (11, 22, 35, 64):
        n = 6
        A = rng.normal(size=(n, 3 * F, F))
        G = np.einsum("sri,srj->sij", A, A)
        truth = np.where(rng.random((n, F)) < 0.3, rng.normal(0, 2, (n, F)), 0.0)
        b = np.einsum("sij,sj->si", G, truth) + rng.normal(0, 0.05, (n, F))
        coef, mask, iters = ops.stlsq(_dl(G, dev), _dl(b, dev), 0.3, 0.5)
        c = coef.cpu().numpy()
        for s in range(n):
            rc, ri, rit = R.stlsq_gram(G[s], b[s], 0.3, 0.5)
            assert np.array_equal(mask.cpu().numpy()[s] != 0, ri), (F, s)
            assert int(iters.cpu().numpy()[s]) == rit
            np.testing.assert_allclose(c[s], rc, rtol=1e-9, atol=1e-10)


def test_joint_gram_matches_oracle(dev, c_coll_ml):
    from insite_amd import ops
    from insite_amd.library import polynomial_library
    tr = c_coll_ml["train"]
    x, inputs, stat, rows = R.de_format_joint(tr.data, tr.scaling_params)
    lib = polynomial_library(2, 2, True, n_inputs=1)
    assert lib.n_terms == 11 and lib.get_feature_names()[2] == "u0"
    code = inputs[..., 0].astype(np.int8)
    for layout in ("patient", "time"):
        xt = _dl(x if layout == "patient" else x.T, dev)
        ct = _dl(code if layout == "patient" else code.T, dev)
        G, b = ops.gen_gram(xt, _dl(stat, dev), _dl(rows, dev, torch.int32), R.STANDARD_DT, lib, step_in=ct,
                            layout=layout)
        Z, Y = R.build_regression_joint(x, inputs, stat, rows, R.STANDARD_DT)
        th = R.eval_library(lib.exps.astype(np.int64), Z)
        np.testing.assert_allclose(G.cpu().numpy()[0], th.T @ th, rtol=1e-11, atol=1e-9)
        np.testing.assert_allclose(b.cpu().numpy()[0], th.T @ Y, rtol=1e-11, atol=1e-9)


@pytest.mark.parametrize("fd", ["order1", "smoothed1"])
def test_joint_gram_two_inputs_order1_matches_oracle(dev, fd):
    """The cancer_sim / EQ_5 joint layout: two binary treatment inputs (chemo, radio), one static, FD order 1
    (or savgol(2,1) + order 1) over the whole row (no segment split in joint mode, pkpd/utils.py:656-672)."""
    from insite_amd import ops
    from insite_amd.library import polynomial_library
    rng = np.random.default_rng(5)
    N, T = 300, 40
    x = 20 * np.exp(-0.05 * np.arange(T)[None, :] * rng.uniform(0.5, 2, (N, 1))) + rng.normal(0, 0.01, (N, T))
    inputs = (rng.random((N, T, 2)) < 0.3).astype(np.float64)
    stat = rng.normal(0, 1, (N, 1))
    rows = rng.integers(2, T + 1, N)
    lib = polynomial_library(1, 2, True, n_inputs=2)
    code = (inputs[..., 0] + 2 * inputs[..., 1]).astype(np.int8)
    G, b = ops.gen_gram(_dl(x, dev), _dl(stat, dev), _dl(rows, dev, torch.int32), 0.1, lib, step_in=_dl(code, dev),
                        fd=fd)
    Z, Y = R.build_regression_joint(x, inputs, stat, rows, 0.1, fd=fd)
    th = R.eval_library(lib.exps.astype(np.int64), Z)
    np.testing.assert_allclose(G.cpu().numpy()[0], th.T @ th, rtol=1e-11, atol=1e-9)
    np.testing.assert_allclose(b.cpu().numpy()[0], th.T @ Y, rtol=1e-11, atol=1e-9)


def _args(eq, *extra):
    from insite_amd import config as C
    return C.compose(["+backbone=sindy", "+dataset=pkpd_sim", f"dataset.equation_str={eq}", f"model.dataset_name={eq}",
                      "model.sindy_threshold=0.1", "model.sindy_alpha=0.5", "model.lam=10.0", *extra])


def test_plugin_joint_model_matches_oracle(dev, c_coll_ml):
    from insite_amd.sindy import SINDY
    m = SINDY(_args("EQ_4_C", "model.joint_model=true", "dataset.treatment_mode=multilabel"), device=dev)
    m.fit(c_coll_ml["train"], c_coll_ml["val"])
    ref = R.sindy_pipeline(c_coll_ml, dt=R.STANDARD_DT, joint_model=True)
    assert m.joint_coefs.shape == (1, 11)
    assert np.array_equal(m.joint_coefs != 0, ref["joint_coefs"] != 0)
    assert np.max(np.abs(m.joint_coefs - ref["joint_coefs"])) < 1e-8
    assert m.global_equation_string.startswith("Joint Model: x_dot = ")
    o, a, last = m.get_normalised_masked_rmse(c_coll_ml["test_cf_one_step"], one_step_counterfactual=True)
    np.testing.assert_allclose([o, a, last], [ref["encoder_test_rmse_orig"], ref["encoder_test_rmse_all"],
                                              ref["encoder_test_rmse_last"]], rtol=1e-8)
    r = m.get_normalised_n_step_rmses(c_coll_ml["test_cf_treatment_seq"])
    np.testing.assert_allclose(r, [ref[f"decoder_test_rmse_{k + 2}-step"] for k in range(len(r))], rtol=1e-8)


def test_plugin_degree4_ablation_matches_oracle(dev, c_coll):
    from insite_amd.sindy import SINDY
    m = SINDY(_args("EQ_4_C", "model.ablation_more_complex_basis_functions=true"), device=dev)
    m.fit(c_coll["train"], c_coll["val"])
    ref = R.sindy_pipeline(c_coll, dt=R.STANDARD_DT, degree=4, interaction_only=False)
    assert m.joint_coefs.shape == (2, 35)
    assert np.array_equal(m.joint_coefs != 0, ref["joint_coefs"] != 0)
    np.testing.assert_allclose(m.joint_coefs, ref["joint_coefs"], rtol=1e-6, atol=1e-9)
    o, a, last = m.get_normalised_masked_rmse(c_coll["test_cf_one_step"], one_step_counterfactual=True)
    np.testing.assert_allclose([o, a, last], [ref["encoder_test_rmse_orig"], ref["encoder_test_rmse_all"],
                                              ref["encoder_test_rmse_last"]], rtol=1e-6)
