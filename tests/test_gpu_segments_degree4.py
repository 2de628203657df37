"""The degree-4 library on the treatment-segment datasets (ABLATION_MORE_COMPLEX_BASIS_FUNCTIONS over
cancer_sim / EQ_5: PolynomialLibrary(degree=4, interaction_only=False), sindy.py:185-186; run.py:96-104,
208) through insite_gen_gram_segments_f64 (per-arm power moments of the segment rows, insite_gen.hip)
against oracle/segments_ref.py (explicit Theta over the literal segment walk), on the reference's own
cancer_sim cohort (oracle/cancer_sim_ref.py, seed 1): per-arm Gram/moments to rtol 1e-9 (x reaches 1150,
so G spans x^8 ~ 1e24), both layouts and both derivative methods; the plugin end to end (fit -> 4-arm
polynomial rollout) against the oracle rollout of the fitted model."""
import warnings

import numpy as np
import pytest
import torch

from oracle import cancer_sim_ref as CS
from oracle import insite_ref as R
from oracle import segments_ref as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cohort():
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        coll = CS.make_collection(1, {"train": 400, "val": 20, "test": 10}, with_tests=False)
    tr = coll["train"]
    return coll, CS.de_format_segments(tr.data, tr.scaling_params)


@pytest.mark.parametrize("layout", ["patient", "time"])
@pytest.mark.parametrize("fd", ["order1", "smoothed1"])
def test_gen_gram_segments_matches_oracle(dev, cohort, layout, fd):
    from insite_amd import ops
    from insite_amd.library import polynomial_library
    _, (x, u, arm, sl) = cohort
    lib = polynomial_library(1, 4, False)
    G_ref, b_ref, _ = S.gram_segments(x, u, arm, sl, R.STANDARD_DT, lib.exps.astype(np.int64), fd=fd)
    if layout == "patient":
        xd, ad = torch.tensor(x, device=dev), torch.tensor(arm.astype(np.int8), device=dev)
    else:
        xd = torch.tensor(np.ascontiguousarray(x.T), device=dev)
        ad = torch.tensor(np.ascontiguousarray(arm.T.astype(np.int8)), device=dev)
    G, b = ops.gen_gram_segments(xd, ad, torch.tensor(sl.astype(np.int32), device=dev),
                                 torch.tensor(np.ascontiguousarray(u), device=dev), R.STANDARD_DT, lib, fd=fd,
                                 layout=layout)
    torch.cuda.synchronize()
    np.testing.assert_allclose(G.cpu().numpy(), G_ref, rtol=1e-9, atol=0)
    np.testing.assert_allclose(b.cpu().numpy(), b_ref, rtol=1e-9, atol=1e-9 * np.abs(b_ref).max())


def test_plugin_degree4_segments_end_to_end(dev):
    """+ablation_more_complex_basis_functions on a 4-arm segment dataset: the GPU's STLSQ on the GPU Gram
    equals the oracle's Gram-form STLSQ on the oracle Gram, and the 4-arm polynomial rollout equals the
    oracle's literal RHS.  A unit-scale synthetic cohort (segments_ref.synthetic_cohort): on the reference's
    cancer_sim cohort (x up to 1150, G up to ~1e24) the degree-4 ridge system is numerically singular --
    sklearn's ridge then falls back to an SVD solve, which the GPU STLSQ does not restate (it reports the
    non-positive-definite system as LinAlgError)."""
    from insite_amd.sindy import SINDY
    from test_gpu_segments import _Subset
    rng = np.random.default_rng(5)
    x, u, arm, sl = S.synthetic_cohort(400, 60, rng, switch_p=0.1, noise=0.01, dt=1 / 6, coef=S.TRUE_COEF_U1,
                                       n_statics=1, min_len=20)
    args = {"model": {"dataset_name": "cancer_sim", "dim_treatments": 4, "dim_static_features": 1,
                      "dim_outcomes": 1, "sindy_threshold": 0.001, "sindy_alpha": 0.5,
                      "ablation_more_complex_basis_functions": True},
            "dataset": {"projection_horizon": 5}, "exp": {"unscale_rmse": True, "percentage_rmse": True}}
    m = SINDY(args, device=dev)
    ds = _Subset(x, u, arm, sl)
    m.fit(ds)
    assert m.library.n_terms == 15 and m.joint_coefs.shape == (4, 15)
    assert m.global_equation_string.count("Treatment ") == 4
    ex = m.library.exps.astype(np.int64)
    G_ref, b_ref, _ = S.gram_segments(x, u, arm, sl, 1 / 6, ex)
    for k in range(4):
        c_ref, ind_ref, _ = R.stlsq_gram(G_ref[k], b_ref[k], 1e-3, 0.5)
        assert np.array_equal(m.joint_coefs[k] != 0, ind_ref), k
        # the degree-4 normal equations are ill-conditioned (cond 1e11..3e13 on this cohort): coefficient
        # agreement is bounded by cond x eps x |c| (up to ~1e-1 here), so the GPU solution is checked as what it
        # is -- the unbiased least-squares minimiser on the support: the same objective to 1e-9 relative (a
        # wrong support or solve moves it by O(1)), evaluated on the oracle's Gram
        c = m.joint_coefs[k]
        obj = lambda v: v @ G_ref[k] @ v - 2.0 * b_ref[k] @ v
        assert abs(obj(c) - obj(c_ref)) <= 1e-9 * max(1.0, abs(obj(c_ref))), k
    p = m.get_predictions(ds)[..., 0]
    y_ref = R.rollout(x[:, 0], u, arm, m.joint_coefs, ex, 1 / 6, "euler5")
    fin = np.isfinite(y_ref)
    assert np.array_equal(np.isfinite(p), fin)
    np.testing.assert_allclose(p[fin], y_ref[fin], rtol=1e-9, atol=1e-9)
