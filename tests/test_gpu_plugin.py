"""GPU: the SINDY plugin end to end (fit -> predictions -> metrics) against the oracle pipeline
(oracle.insite_ref.sindy_pipeline = train_sindy.main restated), and run.py's driver.

Tolerances (BASELINE.json north star): identical support, coefficient L-inf < 1e-8, fp64
trajectory RMSE <= 1e-6; the RMSE metrics agree to 1e-9 relative.
"""
import numpy as np
import pytest
import torch

from oracle import insite_ref as R

pytestmark = pytest.mark.gpu


def _args(eq):
    from insite_amd import config as C
    return C.compose(["+backbone=sindy", "+dataset=pkpd_sim", f"dataset.equation_str={eq}", f"model.dataset_name={eq}",
                      "model.sindy_threshold=0.1", "model.sindy_alpha=0.5", "model.lam=10.0"])


@pytest.fixture(scope="module", params=["EQ_4_A", "EQ_4_C"])
def case(request):
    eq = request.param
    coll = R.make_collection(eq, {"train": 300, "val": 20, "test": 20}, seq_length=60, seed=0)
    ref = R.sindy_pipeline(coll, threshold=0.1, alpha=0.5)
    return eq, coll, ref


def test_plugin_fit_matches_oracle(dev, case):
    from insite_amd.sindy import SINDY
    eq, coll, ref = case
    m = SINDY(_args(eq), device=dev)
    m.fit(coll["train"], coll["val"])
    assert np.array_equal(m.joint_coefs != 0, ref["joint_coefs"] != 0)
    assert np.max(np.abs(m.joint_coefs - ref["joint_coefs"])) < 1e-8
    # the string carries 17 significant digits: the terms must match exactly, the values to 1e-8
    assert _terms(m.global_equation_string) == _terms(ref["global_equation_string"])


def _terms(s):
    return [[t.split("*", 1)[1] for t in arm.split("= ", 1)[1].split("+")[1:]] for arm in s.split(" | ")]


def test_plugin_predictions_and_metrics_match_oracle(dev, case):
    from insite_amd.sindy import SINDY
    eq, coll, ref = case
    m = SINDY(_args(eq), device=dev)
    m.fit(coll["train"])
    m.joint_coefs = ref["joint_coefs"].copy()            # evaluate the identical model
    m._coef_dev = torch.as_tensor(np.where(np.abs(ref["joint_coefs"]) > 1e-3, ref["joint_coefs"], 0.0), device=dev)
    one = coll["test_cf_one_step"]
    p = m.get_predictions(one)
    assert p.shape == one.data["outputs"].shape
    prev, stat = R.unscale_inputs(one.data, one.scaling_params)
    arms = np.argmax(one.data["current_treatments"], axis=-1)
    y_ref = R.rollout(prev[:, 0], stat, arms, ref["joint_coefs"], R.poly_library(3, 2, True), 10.0 / 60)
    sp = one.scaling_params
    y = p[..., 0] * sp["output_stds"] + sp["output_means"]
    assert np.sqrt(np.mean((y - y_ref) ** 2)) <= 1e-6
    o, a, last = m.get_normalised_masked_rmse(one, one_step_counterfactual=True)
    np.testing.assert_allclose([o, a, last], [ref["encoder_test_rmse_orig"], ref["encoder_test_rmse_all"],
                                              ref["encoder_test_rmse_last"]], rtol=1e-9)
    seqs = coll["test_cf_treatment_seq"]
    r = m.get_normalised_n_step_rmses(seqs)
    np.testing.assert_allclose(r, [ref[f"decoder_test_rmse_{k + 2}-step"] for k in range(len(r))], rtol=1e-9)
    ar = m.get_autoregressive_predictions(seqs)
    assert ar.shape == seqs.data_processed_seq["outputs"].shape


def test_log_anchor_eq4c_rmse_last(dev):
    """The reference log's one-step counterfactual RMSE for SINDy on EQ_4_C is 0.1354 (1000 train
    patients; final_with_insite.txt:182); a cohort of the same size lands near it."""
    from insite_amd.sindy import SINDY
    from insite_amd import pkpd
    coll = pkpd.dataset_collection("EQ_4_C", {"train": 1000, "val": 100, "test": 100}, seed=0, device=dev)
    m = SINDY(_args("EQ_4_C"), coll, device=dev)
    m.fit(coll.train_f, coll.val_f)
    sup = [list(np.nonzero(c)[0]) for c in m.joint_coefs]
    assert sup == [[4], [1, 5]]
    _, _, last = m.get_normalised_masked_rmse(coll.test_cf_one_step, one_step_counterfactual=True)
    assert 0.05 < last < 0.3


def test_run_driver_end_to_end(dev):
    import run
    from insite_amd import config as C
    args = C.compose(C.run_overrides(C.driver_config(), "EQ_4_A", "sindy", 0, 2)
                     + ["dataset.num_patients.train=200", "dataset.num_patients.val=10", "dataset.num_patients.test=10"])
    r = run.train_sindy_main(args, "EQ_4_A", device=dev)
    for k in ("encoder_test_rmse_all", "encoder_test_rmse_orig", "encoder_test_rmse_last",
              "decoder_test_rmse_2-step", "decoder_test_rmse_6-step", "global_equation_string"):
        assert k in r
    assert np.isfinite(r["encoder_test_rmse_last"]) and r["fine_tuned"] is False
    assert r["global_equation_string"].startswith("Treatment 0: x_dot = +-1.0")


def test_run_one_log_keys_match_reference(dev):
    """run.py's per-run dict carries the reference's keys in its logged order (reference run.py:305-306 +
    run_exp_wrapper_outer; results/2_main_table/final_with_insite.txt:126): ..., 'global_equation_string',
    'fine_tuned', 'method', 'seed', 'seconds_taken', 'errored', 'dataset_name', 'method_name', 'domain_conf'."""
    import run
    from insite_amd import config as C
    drv = C.driver_config()
    r = run.run_one(drv, "EQ_4_A", "sindy", 0, 2.0, extra=["dataset.num_patients.train=100",
                                                             "dataset.num_patients.val=10",
                                                             "dataset.num_patients.test=10"], device=dev)
    keys = list(r)
    assert keys[-9:] == ["global_equation_string", "fine_tuned", "method", "seed", "seconds_taken", "errored",
                         "dataset_name", "method_name", "domain_conf"]
    assert r["method"] == "sindy" and r["errored"] is False and r["seconds_taken"] > 0
