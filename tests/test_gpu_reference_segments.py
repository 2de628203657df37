"""GPU parity against REFERENCE-HELD OUTPUTS for the treatment-segment family (F4): the reference's own
cancer_sim and EQ_5_B..D cohorts (oracle/cancer_sim_ref.py, numpy legacy-RNG draws restated; the oracle
itself reproduces the logs in tests/test_cancer_sim_reference.py) through the MI355X path must reproduce
the published runs ``results/2_main_table/final_with_insite.txt:6, 54, 78, 102`` (SINDy) -- discovered
equations to L-inf < 1e-10 relative (north star < 1e-8) with identical support, every RMSE metric to 1e-9
relative -- both through the plugin end to end (SINDY.fit -> predictions -> metrics) and through the raw
C ABI (insite_sindy_fit_segments_f64, both HBM layouts).  EQ_5 cohorts carry two statics (patient type and
the t = 0 chemo dosage, include_continuous_treatment; train_sindy.py:41-48), so their library has 7 columns,
the u1 ones exactly zero.  The INSITE runs (4-arm per-row BFGS refinement, insite_refine_arms_f64) are
checked against the oracle restatement per row and through committed oracle metrics."""
import json
import os
import warnings

import numpy as np
import pytest
import torch

from oracle import cancer_sim_ref as CS

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ANCHORS = json.load(open(os.path.join(HERE, "golden", "reference_log_anchors.json")))
METRICS = ["encoder_test_rmse_orig", "encoder_test_rmse_all", "encoder_test_rmse_last"] + \
          [f"decoder_test_rmse_{k}-step" for k in range(2, 7)]


def n_statics(eq):
    return 1 if eq == "cancer_sim" else 2


def names_of(U):
    from insite_amd.library import polynomial_library
    return list(polynomial_library(U, 2, True).get_feature_names())


def logged_coefs(eq_string, names):
    parts = eq_string.split(" | ")
    out = np.zeros((len(parts), len(names)))
    for a, part in enumerate(parts):
        for term in part.split("= ", 1)[1].split("+")[1:]:
            c, name = term.split("*", 1)
            out[a, names.index(name.replace("*", " "))] = float(c)
    return out


def _args(eq, backbone="sindy"):
    from insite_amd import config as C
    a = C.compose([f"+backbone={backbone}", "+dataset=pkpd_sim", "model.sindy_threshold=0.001",
                   "model.sindy_alpha=0.5", "model.lam=10.0"])
    # dim_static_features as train_sindy.py:48 sets it from the processed data
    a["model"].update({"dataset_name": eq, "dim_treatments": 4, "dim_static_features": n_statics(eq),
                       "dim_outcomes": 1})
    return a


@pytest.fixture(scope="module", params=["cancer_sim", "EQ_5_B", "EQ_5_C", "EQ_5_D"])
def case(request):
    eq = request.param
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        return eq, CS.make_collection(1, equation=None if eq == "cancer_sim" else eq)


def _metrics(m, coll):
    o, a, last = m.get_normalised_masked_rmse(coll["test_cf_one_step"], one_step_counterfactual=True)
    got = {"encoder_test_rmse_orig": o, "encoder_test_rmse_all": a, "encoder_test_rmse_last": last}
    r = m.get_normalised_n_step_rmses(coll["test_cf_treatment_seq"])
    got.update({f"decoder_test_rmse_{k + 2}-step": v for k, v in enumerate(r)})
    return got


def test_plugin_reproduces_logged_segment_run(dev, case):
    from insite_amd.sindy import SINDY
    eq, coll = case
    anchor = ANCHORS[f"{eq}/sindy"]
    ref = logged_coefs(anchor["global_equation_string"], names_of(n_statics(eq)))
    m = SINDY(_args(eq), device=dev)
    m.fit(coll["train"], coll["val"])
    assert np.array_equal(m.joint_coefs != 0, ref != 0)
    assert np.max(np.abs(m.joint_coefs - ref) / np.maximum(1.0, np.abs(ref))) < 1e-10
    got = _metrics(m, coll)
    for k in METRICS:
        assert got[k] == pytest.approx(anchor[k], rel=1e-9), k


@pytest.mark.parametrize("layout", ["patient", "time"])
def test_abi_segment_discovery_reproduces_logged_equation(dev, case, layout):
    from insite_amd import ops
    from insite_amd.library import polynomial_library
    from oracle import insite_ref as R
    eq, coll = case
    tr = coll["train"]
    x, u, arm, sl = CS.de_format_segments(tr.data, tr.scaling_params)
    if layout == "patient":
        xd, ad = torch.tensor(x, device=dev), torch.tensor(arm.astype(np.int8), device=dev)
    else:
        xd = torch.tensor(np.ascontiguousarray(x.T), device=dev)
        ad = torch.tensor(np.ascontiguousarray(arm.T.astype(np.int8)), device=dev)
    coef, mask, _, _, _ = ops.sindy_fit_segments(xd, ad, torch.tensor(sl.astype(np.int32), device=dev),
                                                 torch.tensor(np.ascontiguousarray(u), device=dev), R.STANDARD_DT,
                                                 polynomial_library(u.shape[1], 2, True), 1e-3, 0.5, layout=layout)
    ref = logged_coefs(ANCHORS[f"{eq}/sindy"]["global_equation_string"], names_of(u.shape[1]))
    c = coef.cpu().numpy()
    assert np.array_equal(mask.cpu().numpy() != 0, ref != 0)
    assert np.max(np.abs(c - ref) / np.maximum(1.0, np.abs(ref))) < 1e-10


ORACLE_INSITE = json.load(open(os.path.join(HERE, "golden", "segment_insite_oracle.json")))


@pytest.mark.parametrize("subset,tau", [("test_cf_one_step", 1), ("test_cf_treatment_seq", 5)])
def test_insite_segment_rows_match_oracle(dev, case, subset, tau):
    """INSITE on the 4-arm datasets (sindy.py:489-551 non-joint branches): the GPU refinement of every row
    (insite_refine_arms_f64 through ops.insite_refine) against the oracle's BFGS restatement
    (oracle/insite_refine_ref.py) on a fixed sample of rows, first and last included: the same status and
    iteration count, predictions to rtol 1e-9."""
    from insite_amd import ops
    from insite_amd.library import polynomial_library
    from oracle import insite_ref as R
    from oracle import insite_refine_ref as Q
    eq, coll = case
    pipe = CS.sindy_pipeline(coll)
    c0, exps = pipe["joint_coefs"], pipe["exps"]
    sub = coll[subset]
    U = sub.data["static_features"].shape[-1]
    prev, st = R.unscale_inputs(sub.data, sub.scaling_params, 1, U)
    if U >= 2:                                 # the EQ_5 refinement's u1 = static_features[0] (sindy.py:536)
        st = np.repeat(st[:, :1], U, axis=1)
    arms = np.argmax(sub.data["current_treatments"], axis=-1)
    sl = sub.data["sequence_lengths"].astype(np.int64)
    preds, _, status, iters = ops.insite_refine(
        torch.tensor(prev, device=dev), torch.tensor(arms.astype(np.int8), device=dev), torch.tensor(st, device=dev),
        torch.tensor(sl.astype(np.int32), device=dev), c0, polynomial_library(U, 2, True), R.STANDARD_DT, 10.0, tau)
    preds, status, iters = preds.cpu().numpy(), status.cpu().numpy(), iters.cpu().numpy()
    N = prev.shape[0]
    rows = np.unique(np.concatenate([[0, N - 1], np.random.default_rng(3).choice(N, 160, replace=False)]))
    for i in rows:
        p, _, s, k = Q.refine_patient(prev[i], arms[i], st[i], int(sl[i]), c0, exps, R.STANDARD_DT, 10.0, tau)
        assert int(status[i]) == int(s), (i, status[i], s)
        if s >= 0:
            assert int(iters[i]) == int(k), (i, iters[i], k)
        np.testing.assert_allclose(preds[i], p, rtol=1e-9, atol=1e-9 * np.max(np.abs(p)), err_msg=f"row {i}")


# Published INSITE runs vs the restatement ("INSITE on the 4-arm and joint models"): the published runs
# are not reproducible by the restated algorithm (the round-5 stopping-control sweep moves none of the gaps); every
# metric's gap is FROZEN in tests/golden/insite_published_gap.json and asserted to 5e-4 absolute, so a regression that
# moves the GPU path (or the oracle) either way fails.
GAP = json.load(open(os.path.join(HERE, "golden", "insite_published_gap.json")))


def _off_gap(key, rel):
    return {k: (v, GAP["gap"][key][k]) for k, v in rel.items() if abs(v - GAP["gap"][key][k]) > GAP["tolerance_abs"]}


def test_insite_plugin_segment_metrics(dev, case):
    """The plugin end to end (SINDY.fit -> refined predictions -> metrics, insite: true) on the reference's
    cohorts equals the oracle restatement's metrics (tests/golden/segment_insite_oracle.json, made by the
    committed make_segment_insite_oracle.py) to 1e-9 relative, and differs from the PUBLISHED INSITE
    runs (final_with_insite.txt:2362-2382) by exactly the frozen per-metric gap (insite_published_gap.json: cancer_sim
    and EQ_5_C within 1e-3, EQ_5_B / D up to 3.7 %; the published runs' in-window fits are looser than the
    restatement's: DESIGN.md §3)."""
    from insite_amd.sindy import SINDY
    eq, coll = case
    ref = ORACLE_INSITE[eq]["oracle"]
    m = SINDY(_args(eq, "insite"), device=dev)
    m.fit(coll["train"], coll["val"])
    got = _metrics(m, coll)
    anchor = ANCHORS[f"{eq}/insite"]
    rel = {k: got[k] / anchor[k] - 1 for k in METRICS}
    print(eq, "log rel diff", {k: f"{v:+.2e}" for k, v in rel.items()})
    bad = {k: (got[k], ref[k]) for k in METRICS if got[k] != pytest.approx(ref[k], rel=1e-9)}
    assert not bad, bad
    far = _off_gap(eq, rel)
    assert not far, far


def test_insite_plugin_joint_one_ode_metrics(dev):
    """INSITE on the one-ODE ablation (run.py:198-201: joint_model + multilabel, the np.random.seed(10) cohort of
    the dataset cache): the plugin's refined metrics equal the oracle restatement's (segment_insite_oracle.json)
    to 1e-9 and sit at the frozen gap from the published joint INSITE runs (one_big_ode.txt:6; the restatement fits
    tighter, up to 21 % on the 2-step metric: DESIGN.md §3)."""
    from insite_amd import config as C
    from insite_amd.sindy import SINDY
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        coll = CS.make_collection(10, treatment_mode="multilabel")
    a = C.compose(["+backbone=insite", "+dataset=pkpd_sim", "model.sindy_threshold=0.001", "model.sindy_alpha=0.5",
                   "model.lam=10.0", "model.joint_model=true", "dataset.treatment_mode=multilabel"])
    a["model"].update({"dataset_name": "cancer_sim", "dim_treatments": 2, "dim_static_features": 1,
                       "dim_outcomes": 1})
    m = SINDY(a, device=dev)
    m.fit(coll["train"], coll["val"])
    got = _metrics(m, coll)
    key = "ABLATION_ONE_ODE/cancer_sim"
    ref = ORACLE_INSITE[key]["oracle"]
    anchor = ANCHORS["ABLATION_ONE_ODE/cancer_sim/insite/1"]
    rel = {k: got[k] / anchor[k] - 1 for k in METRICS}
    print("one-ODE joint INSITE log rel diff", {k: f"{v:+.2e}" for k, v in rel.items()})
    bad = {k: (got[k], ref[k]) for k in METRICS if got[k] != pytest.approx(ref[k], rel=1e-9)}
    assert not bad, bad
    far = _off_gap(key, rel)
    assert not far, far


def test_plugin_joint_one_ode_reproduces_log(dev):
    """The one-ODE ablation (run.py:198-201, joint_model + multilabel treatments) through the plugin on the GPU
    (general one-state Gram + STLSQ, folded per-combination rollout) on the logged cohort (np.random.seed(10),
    tests/test_cancer_sim_reference.py::test_one_ode_joint_model_equals_log): the 16-digit equation of
    results/ablation/one_ode/build_tables/...one_big_ode.txt:10 to 1e-10 relative and every metric to 1e-9."""
    from insite_amd import config as C
    from insite_amd.sindy import SINDY
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        coll = CS.make_collection(10, treatment_mode="multilabel")
    a = C.compose(["+backbone=sindy", "+dataset=pkpd_sim", "model.sindy_threshold=0.001", "model.sindy_alpha=0.5",
                   "model.joint_model=true", "dataset.treatment_mode=multilabel"])
    a["model"].update({"dataset_name": "cancer_sim", "dim_treatments": 2, "dim_static_features": 1,
                       "dim_outcomes": 1})
    m = SINDY(a, device=dev)
    m.fit(coll["train"], coll["val"])
    anchor = ANCHORS["ABLATION_ONE_ODE/cancer_sim/sindy/1"]
    names = ["1", "x0", "u0", "u1", "u2", "x0 u0", "x0 u1", "x0 u2", "u0 u1", "u0 u2", "u1 u2"]
    parts = anchor["global_equation_string"].split("= ", 1)[1].split("+")[1:]
    ref = np.zeros(len(names))
    for term in parts:
        c, name = term.split("*", 1)
        ref[names.index(name.replace("*", " "))] = float(c)
    got = np.asarray(m.joint_coefs)[0]
    assert np.array_equal(got != 0, ref != 0)
    assert np.max(np.abs(got - ref) / np.maximum(1.0, np.abs(ref))) < 1e-10
    res = _metrics(m, coll)
    for k in METRICS:
        assert res[k] == pytest.approx(anchor[k], rel=1e-9), k
