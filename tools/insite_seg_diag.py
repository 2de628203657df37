"""Diagnostic: INSITE on the reference's cancer_sim / EQ_5 cohorts vs the published INSITE runs, with the
status-3 (zoom failed) rows kept (default) or reverted (sindy.py:628-631 literal).  Prints the metrics'
relative errors and the BFGS status histogram of the tau-step set."""
import json
import os
import sys
import warnings

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd")]
from oracle import cancer_sim_ref as CS  # noqa: E402
from insite_amd import config as C  # noqa: E402
from insite_amd.sindy import SINDY  # noqa: E402

ANCHORS = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_log_anchors.json")))
METRICS = ["encoder_test_rmse_orig", "encoder_test_rmse_all", "encoder_test_rmse_last"] + \
          [f"decoder_test_rmse_{k}-step" for k in range(2, 7)]
dev = torch.device("cuda:0")
for eq in sys.argv[1:] or ["cancer_sim"]:
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        coll = CS.make_collection(1, equation=None if eq == "cancer_sim" else eq)
    for revert in (False, True):
        a = C.compose(["+backbone=insite", "+dataset=pkpd_sim", "model.sindy_threshold=0.001", "model.sindy_alpha=0.5",
                       "model.lam=10.0", f"model.insite_revert_on_zoom_fail={str(revert).lower()}"])
        a["model"].update({"dataset_name": eq, "dim_treatments": 4, "dim_static_features": 1, "dim_outcomes": 1})
        m = SINDY(a, device=dev)
        m.fit(coll["train"], coll["val"])
        o, al, last = m.get_normalised_masked_rmse(coll["test_cf_one_step"], one_step_counterfactual=True)
        st1 = m.insite_status.cpu().numpy()
        got = {"encoder_test_rmse_orig": o, "encoder_test_rmse_all": al, "encoder_test_rmse_last": last}
        r = m.get_normalised_n_step_rmses(coll["test_cf_treatment_seq"])
        st5 = m.insite_status.cpu().numpy()
        got.update({f"decoder_test_rmse_{k + 2}-step": v for k, v in enumerate(r)})
        anc = ANCHORS[f"{eq}/insite"]
        err = {k: float(got[k] / anc[k] - 1) for k in METRICS}
        print(json.dumps({"eq": eq, "revert": revert, "rel_err": err,
                          "status_one_step": {int(s): int((st1 == s).sum()) for s in np.unique(st1)},
                          "status_tau_step": {int(s): int((st5 == s).sum()) for s in np.unique(st5)}}))
