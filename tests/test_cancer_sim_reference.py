"""Parity against REFERENCE-HELD OUTPUTS for the treatment-segment family: the
reference's own cancer_sim and EQ_5_* cohorts, regenerated bit for bit (oracle/cancer_sim_ref.py: the
Geng tumour simulator and its continuous EQ_5 variant restated with numpy's legacy RandomState draw order,
np.random.seed(1)), through the oracle pipeline (segment split, FD order 1, 4-arm STLSQ, Euler-5 4-arm
rollout, the reference's metrics) must reproduce the published runs
``results/2_main_table/final_with_insite.txt:6`` (cancer_sim), ``:54, :78, :102`` (EQ_5_B..D):
16-digit equations to 1e-10 and every RMSE metric to 1e-11 relative.

EQ_5 runs go through ``process_data_multi(include_continuous_treatment=True)`` (train_sindy.py:41-42): the
chemo dosage is a third covariate, so the statics are [patient type, chemo dosage at t = 0] and the library
over (x0, u0, u1) has 7 columns; the factual dosage at t = 0 is 0, the u1 columns are zero and their
coefficients exactly 0 -- the logged strings omit |c| <= 1e-3 terms (pkpd/utils.py:387-391), so the log
shows 4 terms per arm.

EQ_5_A (``:30``): its single patient type makes the static column u0 == 1, so the library columns
{1, u0} and {x0, x0 u0} coincide and pysindy's unbias lstsq is singular.  Arms 1 and 2 reproduce the log
(where the logged solve landed on the minimum-norm split, equal halves, as here); arms 0 and 3 are logged
as +-1.4e8 / +-3.8e12 and +-1.7e9 / +-1.8e13 pairs -- rounding artefacts of the noise-free, exactly
singular solve that no restatement can pin.  EQ_5_A's metrics depend on them and are not checked.
"""
import json
import os
import warnings

import numpy as np
import pytest

from oracle import cancer_sim_ref as CS
from oracle import insite_ref as R

HERE = os.path.dirname(os.path.abspath(__file__))
ANCHORS = json.load(open(os.path.join(HERE, "golden", "reference_log_anchors.json")))
NAMES = ["1", "x0", "u0", "x0 u0"]
METRICS = ["encoder_test_rmse_orig", "encoder_test_rmse_all", "encoder_test_rmse_last"] + \
          [f"decoder_test_rmse_{k}-step" for k in range(2, 7)]


def logged_coefs(eq_string, names=NAMES):
    parts = eq_string.split(" | ")
    out = np.zeros((len(parts), len(names)))
    for a, part in enumerate(parts):
        for term in part.split("= ", 1)[1].split("+")[1:]:
            c, name = term.split("*", 1)
            out[a, names.index(name.replace("*", " "))] = float(c)
    return out


@pytest.fixture(scope="module", params=["cancer_sim", "EQ_5_B", "EQ_5_C", "EQ_5_D", "EQ_5_A"])
def pipeline(request):
    eq = request.param
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)     # exp overflow of the recovery test, as in the reference
        coll = CS.make_collection(1, equation=None if eq == "cancer_sim" else eq)
        return eq, coll, CS.sindy_pipeline(coll)


def test_segment_equation_and_metrics_equal_log(pipeline):
    eq, _, res = pipeline
    anchor = ANCHORS[f"{eq}/sindy"]
    names = res["names"]
    ref = logged_coefs(anchor["global_equation_string"], names)
    got = res["joint_coefs"]
    arms = [1, 2] if eq == "EQ_5_A" else [0, 1, 2, 3]
    assert np.array_equal(got[arms] != 0, ref[arms] != 0)
    assert np.max(np.abs(got[arms] - ref[arms]) / np.maximum(1.0, np.abs(ref[arms]))) < 1e-10
    if eq == "EQ_5_A":       # the singular arms 0 / 3: the duplicated columns' halves are equal here
        pair = [names.index("u0"), names.index("x0 u0")]
        np.testing.assert_allclose(got[[0, 3]][:, [0, 1]], got[[0, 3]][:, pair], rtol=1e-9)
        return
    for k in METRICS:
        assert res[k] == pytest.approx(anchor[k], rel=1e-11), k


def test_cohort_layout(pipeline):
    """The collection's shapes and scaling follow SyntheticCancerDataset.process_data (dataset.py:96-185)."""
    eq, coll, _ = pipeline
    tr = coll["train"]
    assert tr.data["outputs"].shape == (1000, 59, 1)
    assert tr.data["current_treatments"].shape == (1000, 59, 4)
    assert np.all(tr.data["current_treatments"].sum(-1) == 1)
    assert coll["test_cf_treatment_seq"].data_processed_seq["outputs"].shape[1:] == (5, 1)
    assert coll["val"].scaling_params["output_means"] == tr.scaling_params["output_means"]
    assert tr.norm_const == pytest.approx(CS.calc_volume(13))
    # EQ_5: statics [patient type, chemo dosage at t = 0] (continuous/dataset.py:112-117, 160-163, 191)
    U = 1 if eq == "cancer_sim" else 2
    assert tr.data["static_features"].shape == (1000, U)
    assert len(tr.scaling_params["input_means"]) == 3 + U
    if U == 2:
        u = CS.de_format_segments(tr.data, tr.scaling_params)[1]
        assert np.all(u[:, 1] == 0.0)           # the factual simulation doses from t = 1 (continuous.py:308)


def test_one_ode_joint_model_equals_log():
    """The one-ODE ablation (run.py:198-201: joint_model, multilabel treatments) on cancer_sim: the published
    runs (results/ablation/one_ode/build_tables/...one_big_ode.txt, identical for exp seeds 1-5 -- the
    collection came from the dataset cache) are the cohort of np.random.seed(10): its joint fit (one library over
    x0, chemo, radio, patient type; FD order 1) reproduces the logged 16-digit equation and every SINDy metric
    (the other seeds tried, 0-5, 42 and 100, miss by 5-50 %)."""
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        coll = CS.make_collection(10, treatment_mode="multilabel")
    res = CS.joint_pipeline(coll)
    anchor = ANCHORS["ABLATION_ONE_ODE/cancer_sim/sindy/1"]
    names = ["1", "x0", "u0", "u1", "u2", "x0 u0", "x0 u1", "x0 u2", "u0 u1", "u0 u2", "u1 u2"]
    ref = logged_coefs(anchor["global_equation_string"], names)[0]
    got = res["joint_coefs"][0]
    assert np.array_equal(got != 0, ref != 0)
    assert np.max(np.abs(got - ref) / np.maximum(1.0, np.abs(ref))) < 1e-10
    for k in METRICS:
        assert res[k] == pytest.approx(anchor[k], rel=1e-11), k


def test_insite_restatement_vs_published_runs_frozen_gap():
    """The restated INSITE refinement (tests/golden/segment_insite_oracle.json, regenerated by the committed
    make_segment_insite_oracle.py) against the PUBLISHED INSITE runs on the bit-identical cohorts: every metric's
    relative gap equals its FROZEN value (tests/golden/insite_published_gap.json, 5e-4 absolute) -- the published
    runs are not reproducible by the restated algorithm (the round-5 stopping-control sweep moves no
    gap), so the gap itself is pinned and a move of either sign fails.  The gap has the recorded shape: the
    published runs' fitted window carries MORE squared error than the restatement's, while their last
    (counterfactual) entry agrees within 1 %."""
    import json
    import os
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    fx = json.load(open(os.path.join(here, "segment_insite_oracle.json")))
    frozen = json.load(open(os.path.join(here, "insite_published_gap.json")))
    tol = frozen["tolerance_abs"]
    assert set(frozen["gap"]) == set(fx)
    for key, gap in frozen["gap"].items():
        rel = fx[key]["log_rel_diff"]
        assert set(rel) == set(gap) and len(rel) == 8, key
        off = {k: (rel[k], gap[k]) for k in gap if abs(rel[k] - gap[k]) > tol}
        assert not off, (key, off)
    for eq in ("cancer_sim", "EQ_5_B", "EQ_5_C", "EQ_5_D"):
        d = fx[eq]["one_step_decomposition"]
        w, last = d["in_window_sse"], d["last_entry_sse"]
        assert w["oracle"] < w["log_implied"] < w["sindy_model"], (eq, w)
        assert abs(last["log_implied"] / last["oracle"] - 1) < 1e-2, (eq, last)


def _refine_rows_eq5(args):
    from oracle import insite_refine_ref as Q
    prev, arms, stat, sl, c0, exps = args
    return [Q.refine_patient(prev[i], arms[i], stat[i], int(sl[i]), c0, exps, R.STANDARD_DT, 10.0, 1)[0]
            for i in range(prev.shape[0])]


def test_insite_restatement_reproduces_fixture_eq5d_one_step():
    """The fixture is the restatement's own output: EQ_5_D's one-step INSITE metrics recomputed live (21,860
    refinements over the host's cores) equal segment_insite_oracle.json to 1e-9 -- so the frozen published-run gap
    above is the live oracle's, not a stale file's."""
    import json
    import os
    from concurrent.futures import ProcessPoolExecutor
    fx = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                     "segment_insite_oracle.json")))["EQ_5_D"]["oracle"]
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        coll = CS.make_collection(1, equation="EQ_5_D")
    pipe = CS.sindy_pipeline(coll)
    one = coll["test_cf_one_step"]
    U = one.data["static_features"].shape[-1]
    prev, st = R.unscale_inputs(one.data, one.scaling_params, 1, U)
    st = np.repeat(st[:, :1], U, axis=1)                    # the EQ_5 refinement's u1 = static_features[0]
    arms = np.argmax(one.data["current_treatments"], axis=-1)
    sl = one.data["sequence_lengths"].astype(np.int64)
    chunks = np.array_split(np.arange(prev.shape[0]), 64)
    with ProcessPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        P = np.stack([p for o in ex.map(_refine_rows_eq5, [(prev[c], arms[c], st[c], sl[c], pipe["joint_coefs"],
                                                               pipe["exps"]) for c in chunks]) for p in o])
    m = R.masked_rmse(P[..., None], one.data["unscaled_outputs"], one.data["active_entries"],
                      CS.TUMOUR_DEATH_THRESHOLD, one_step_counterfactual=True)
    for v, k in zip(m, ["encoder_test_rmse_orig", "encoder_test_rmse_all", "encoder_test_rmse_last"]):
        assert v == pytest.approx(fx[k], rel=1e-9), k
