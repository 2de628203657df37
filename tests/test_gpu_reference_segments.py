"""GPU parity against REFERENCE-HELD OUTPUTS for the treatment-segment family (F4): the reference's own
cancer_sim and EQ_5_B..D cohorts (oracle/cancer_sim_ref.py, numpy legacy-RNG draws restated; the oracle
itself reproduces the logs in tests/test_cancer_sim_reference.py) through the MI355X path must reproduce
the published runs ``results/2_main_table/final_with_insite.txt:6, 54, 78, 102`` (SINDy) -- discovered
equations to L-inf < 1e-10 relative (north star < 1e-8) with identical support, every RMSE metric to 1e-9
relative -- both through the plugin end to end (SINDY.fit -> predictions -> metrics) and through the raw
C ABI (insite_sindy_fit_segments_f64, both HBM layouts); and the INSITE runs (``:2326`` onward, 4-arm
per-row BFGS refinement, insite_refine_arms_f64) to 1e-8 relative."""
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
NAMES = ["1", "x0", "u0", "x0 u0"]
METRICS = ["encoder_test_rmse_orig", "encoder_test_rmse_all", "encoder_test_rmse_last"] + \
          [f"decoder_test_rmse_{k}-step" for k in range(2, 7)]


def logged_coefs(eq_string):
    parts = eq_string.split(" | ")
    out = np.zeros((len(parts), len(NAMES)))
    for a, part in enumerate(parts):
        for term in part.split("= ", 1)[1].split("+")[1:]:
            c, name = term.split("*", 1)
            out[a, NAMES.index(name.replace("*", " "))] = float(c)
    return out


def _args(eq, backbone="sindy"):
    from insite_amd import config as C
    a = C.compose([f"+backbone={backbone}", "+dataset=pkpd_sim", "model.sindy_threshold=0.001",
                   "model.sindy_alpha=0.5", "model.lam=10.0"])
    a["model"].update({"dataset_name": eq, "dim_treatments": 4, "dim_static_features": 1, "dim_outcomes": 1})
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
    ref = logged_coefs(anchor["global_equation_string"])
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
                                                 polynomial_library(1, 2, True), 1e-3, 0.5, layout=layout)
    ref = logged_coefs(ANCHORS[f"{eq}/sindy"]["global_equation_string"])
    c = coef.cpu().numpy()
    assert np.array_equal(mask.cpu().numpy() != 0, ref != 0)
    assert np.max(np.abs(c - ref) / np.maximum(1.0, np.abs(ref))) < 1e-10


def test_insite_plugin_reproduces_logged_segment_run(dev, case):
    """INSITE on the 4-arm datasets (sindy.py:489-551 non-joint branches): per-row BFGS refinement of every
    one-step and tau-step row on the GPU, against the published INSITE runs."""
    from insite_amd.sindy import SINDY
    eq, coll = case
    anchor = ANCHORS[f"{eq}/insite"]
    m = SINDY(_args(eq, "insite"), device=dev)
    m.fit(coll["train"], coll["val"])
    got = _metrics(m, coll)
    bad = {k: (got[k], anchor[k]) for k in METRICS if got[k] != pytest.approx(anchor[k], rel=1e-8)}
    assert not bad, bad
