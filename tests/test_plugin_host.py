"""CPU tests of the plugin's host logic: config composition, SINDY construction and validation,
equation strings, the PK/PD collection layout, DE-format extraction and the tau-step slice.
No kernels run here (the device ops are covered by tests/test_gpu_*.py)."""
import numpy as np
import pytest
import torch

from oracle import insite_ref as R


def _args(**model):
    from insite_amd import config as C
    ov = ["+backbone=sindy", "+dataset=pkpd_sim", "dataset.equation_str=EQ_4_C", "model.dataset_name=EQ_4_C",
          "model.sindy_threshold=0.1", "model.sindy_alpha=0.5", "model.lam=10.0"]
    ov += [f"model.{k}={v}" for k, v in model.items()]
    return C.compose(ov)


def test_compose_groups_and_overrides():
    a = _args()
    assert a["model"]["name"] == "SINDY" and a["model"]["sindy_threshold"] == 0.1
    assert a["dataset"]["equation_str"] == "EQ_4_C" and a["dataset"]["projection_horizon"] == 5
    assert a["exp"]["unscale_rmse"] is True and a["dataset"]["seed"] == 0
    from insite_amd import config as C
    b = C.compose(["+backbone=insite", "exp.seed=3", "+dataset=pkpd_sim"])
    assert b["model"]["insite"] is True and b["dataset"]["seed"] == 3
    with pytest.raises(FileNotFoundError):
        C.compose(["+backbone=crn"])


def test_run_overrides_pick_thresholds_by_dataset():
    from insite_amd import config as C
    drv = C.driver_config()
    ov = C.run_overrides(drv, "EQ_4_D", "sindy", 2, 2)
    a = C.compose(ov)
    assert a["model"]["sindy_threshold"] == 0.1 and a["model"]["lam"] == 10.0
    assert a["dataset"]["num_patients"] == {"train": 1000, "val": 100, "test": 100}
    assert a["exp"]["seed"] == 2 and a["dataset"]["coeff"] == 2
    with pytest.raises(NotImplementedError):
        C.run_overrides(drv, "cancer_sim", "sindy", 0, 2)


def test_sindy_reads_config_and_rejects_unsupported_modes():
    from insite_amd.sindy import SINDY
    m = SINDY(_args(), device="cpu")
    assert (m.sindy_threshold, m.sindy_alpha, m.dt) == (0.1, 0.5, 10.0 / 60)
    assert m.feature_library_names == ["1", "x0", "u0", "u1", "x0 u0", "x0 u1", "u0 u1"]
    assert m.model_type == "sindy_regressor" and m.insite is False
    with pytest.raises(NotImplementedError):
        SINDY(_args(wsindy=True), device="cpu")
    for flag in ("joint_model", "ablation_more_complex_basis_functions"):   # the ablations run (insite_gen.hip) ...
        m2 = SINDY(_args(**{flag: True}), device="cpu")
        assert getattr(m2, flag) is True
        m3 = SINDY(_args(insite=True, **{flag: True}), device="cpu")          # ... and so does their INSITE refinement
        assert m3.insite and getattr(m3, flag)
    m4 = SINDY(_args(ablation_more_complex_basis_functions=True), device="cpu")
    assert m4.library.n_terms == 35 and m4.feature_library_names[4] == "x0^2"
    ins = SINDY(_args(insite=True), device="cpu")   # the INSITE refinement (F2) is on the GPU path
    assert ins.insite is True
    with pytest.raises(RuntimeError):               # refined predictions before fit()
        ins._predict_device(None)
    a = _args(dim_treatments=4, dim_static_features=1)
    a["model"]["dataset_name"] = "cancer_sim"
    seg = SINDY(a, device="cpu")                 # F4: the treatment-segment path
    assert seg.segment_mode and seg.feature_library_names == ["1", "x0", "u0", "x0 u0"]
    a["model"]["insite"] = True
    seg_ins = SINDY(a, device="cpu")             # INSITE on 4 arms: insite_refine_arms_f64
    assert seg_ins.segment_mode and seg_ins.insite
    a = _args()
    a["model"]["dataset_name"] = "mimic3"
    with pytest.raises(NotImplementedError):
        SINDY(a, device="cpu")
    with pytest.raises(ValueError):
        SINDY(_args(integrator="rk45"), device="cpu")
    with pytest.raises(RuntimeError):          # predictions before fit()
        SINDY(_args(), device="cpu")._predict_device(None)


def test_equation_string_matches_oracle_and_quantize():
    from insite_amd.sindy import equation_string, rhs_coefficients
    g = np.load("tests/golden/discovery_eq_4_c.npz")
    names = ["1", "x0", "u0", "u1", "x0 u0", "x0 u1", "u0 u1"]
    assert equation_string(g["coef"], names) == str(g["equation"]) == R.global_equation_string(g["coef"], names)
    c = np.array([[0.0, 0.0005, 0.0, 0.0, -1.23456, 0.0, 0.0]])
    assert equation_string(c, names, quantize=True, round_to=2) == "Treatment 0: x_dot = +-1.23*x0*u0"
    np.testing.assert_array_equal(rhs_coefficients(c, True, 2), [[0, 0, 0, 0, -1.23, 0, 0]])
    np.testing.assert_array_equal(rhs_coefficients(c), [[0, 0, 0, 0, -1.23456, 0, 0]])


def test_de_format_on_host_torch_matches_oracle():
    from insite_amd.sindy import SINDY
    coll = R.make_collection("EQ_4_C", {"train": 50, "val": 2, "test": 2}, seq_length=60, seed=1, with_tests=False)
    tr = coll["train"]
    m = SINDY(_args(), device="cpu")
    x, u, arm, rows = m.de_format(tr)
    xr, ur, ar, rr = R.de_format(tr.data, tr.scaling_params)
    np.testing.assert_array_equal(x.numpy(), xr)
    np.testing.assert_array_equal(u.numpy(), ur)
    np.testing.assert_array_equal(arm.numpy(), ar)
    np.testing.assert_array_equal(rows.numpy(), rr)


def test_tau_slice_matches_oracle():
    from insite_amd.sindy import SINDY
    m = SINDY(_args(), device="cpu")
    pred = torch.arange(6 * 12, dtype=torch.float64).reshape(6, 12)

    class D:
        data = {"sequence_lengths": np.array([12.0, 3.0, 6.0, 1.0, 9.0, 5.0])}
    got = m._slice_device(pred, D()).numpy()
    ref = R.autoregressive_slice(pred.numpy()[..., None], D.data["sequence_lengths"], 5)[..., 0]
    np.testing.assert_array_equal(got, ref)


def test_pkpd_collection_layout_matches_reference_format():
    from insite_amd import pkpd
    c = pkpd.dataset_collection("EQ_4_C", {"train": 40, "val": 5, "test": 4}, seed=0, device="cpu", rng="torch")
    o = R.make_collection("EQ_4_C", {"train": 40, "val": 5, "test": 4}, seq_length=60, seed=0)
    for mine, ref in ((c.train_f, o["train"]), (c.val_f, o["val"]), (c.test_cf_one_step, o["test_cf_one_step"]),
                      (c.test_cf_treatment_seq, o["test_cf_treatment_seq"])):
        for k, v in ref.data.items():
            if k.startswith("hidden_"):
                continue
            assert mine.data[k].shape == v.shape, k
            assert mine.data[k].dtype == v.dtype, k
        assert set(mine.scaling_params) == set(ref.scaling_params)
    for k, v in o["test_cf_treatment_seq"].data_processed_seq.items():
        assert c.test_cf_treatment_seq.data_processed_seq[k].shape == v.shape
    # every subset uses the train scaling
    assert c.test_cf_one_step.scaling_params["output_means"] == c.train_f.scaling_params["output_means"]


def test_pkpd_counterfactual_structure():
    """One-step rows come in pairs that share the history and differ in the last step only
    (treatment flipped at step i); tau-step rows follow one-hot / inverted one-hot plans."""
    from insite_amd import pkpd
    T, tau = 12, 3
    c = pkpd.SyntheticPkpdDatasetCollection(2.0, {"train": 6, "val": 2, "test": 3}, "EQ_4_A", seed=4,
                                            max_seq_length=T, projection_horizon=tau, device="cpu", rng="torch")
    one = {k: v.numpy() for k, v in c.test_cf_one_step.sim.items()}
    V, trt, sl = one["cancer_volume"], one["treatment_application"], one["sequence_lengths"]
    for p in range(3):
        for i in range(T - 1):
            r0, r1 = p * 2 * (T - 1) + 2 * i, p * 2 * (T - 1) + 2 * i + 1
            assert sl[r0] == sl[r1] == i + 1
            np.testing.assert_array_equal(V[r0, : i + 1], V[r1, : i + 1])
            assert trt[r0, i] == 1 - trt[r1, i]
            assert np.all(V[r0, i + 2:] == 0) and np.all(V[r1, i + 2:] == 0)
    seq = {k: v.numpy() for k, v in c.test_cf_treatment_seq.sim.items()}
    trt, sl = seq["treatment_application"], seq["sequence_lengths"]
    plans = np.concatenate([np.eye(tau), 1 - np.eye(tau)])
    for i in range(T - 1):
        for p in range(2 * tau):
            r = i * 2 * tau + p
            assert sl[r] == i + 1 + tau
            np.testing.assert_array_equal(trt[r, i + 1: i + 1 + tau], plans[p])


def test_pkpd_noise_free_trajectory_is_euler5_decay():
    from insite_amd import pkpd
    c = pkpd.SyntheticPkpdDatasetCollection(2.0, {"train": 20, "val": 2, "test": 2}, "EQ_4_A", seed=5,
                                            max_seq_length=30, device="cpu", rng="torch")
    s = {k: v.numpy() for k, v in c.train_f.sim.items()}
    V, a = s["cancer_volume"], s["treatment_application"][:, 0]
    dt = 10.0 / 30
    # EQ_4_A: C_a = c_a (observed statics), no noise
    C = np.where(a == 0, s["observed_static_c_0"], s["observed_static_c_1"])
    ratio = V[:, 1:] / V[:, :-1]
    np.testing.assert_allclose(ratio, np.broadcast_to(((1 - C * dt / 5) ** 5)[:, None], ratio.shape), rtol=1e-12)


def test_pkpd_is_deterministic_per_seed():
    from insite_amd import pkpd
    a = pkpd.dataset_collection("EQ_4_D", {"train": 10, "val": 2, "test": 2}, seed=9, device="cpu", rng="torch")
    b = pkpd.dataset_collection("EQ_4_D", {"train": 10, "val": 2, "test": 2}, seed=9, device="cpu", rng="torch")
    np.testing.assert_array_equal(a.train_f.data["outputs"], b.train_f.data["outputs"])
    c = pkpd.dataset_collection("EQ_4_D", {"train": 10, "val": 2, "test": 2}, seed=10, device="cpu", rng="torch")
    assert not np.array_equal(a.train_f.data["outputs"], c.train_f.data["outputs"])


def test_pkpd_threefry_needs_the_device():
    """rng='threefry' (the default, the reference's draws) runs on the HIP kernel: a CPU device is refused
    loudly rather than served by a host generator."""
    from insite_amd import pkpd
    with pytest.raises(RuntimeError, match="threefry"):
        pkpd.dataset_collection("EQ_4_A", {"train": 4, "val": 2, "test": 2}, seed=1, device="cpu")
    with pytest.raises(ValueError):
        pkpd.subset_rngs("pcg", 1, "train", "cpu")


def test_savgol_rows_matches_scipy():
    """smooth_input_data (INSITE path, sindy.py:557-560): scipy savgol_filter(5, 3, mode='interp')."""
    import torch
    from scipy.signal import savgol_filter
    from insite_amd.sindy import savgol_5_3_rows
    V = np.random.default_rng(0).normal(size=(7, 23))
    got = savgol_5_3_rows(torch.tensor(V)).numpy()
    assert np.allclose(got, savgol_filter(V, 5, 3, axis=1), rtol=1e-12, atol=1e-12)


def test_workspace_kind_is_enforced():
    """A workspace serves one op family: the discovery kernels' zero counter header must never be
    overwritten by an op that writes scratch from offset 0."""
    from insite_amd import ops
    ws = ops.Workspace()
    assert ws.claim("disc") is ws and ws.claim("disc") is ws
    with pytest.raises(ValueError, match="separate Workspace"):
        ws.claim("scratch")
    ws2 = ops.Workspace("scratch")
    with pytest.raises(ValueError):
        ops._plan_ws(ws2)
    assert ops._plan_ws(None).kind == "disc"


def test_failed_run_keeps_its_seed():
    """run_exp_wrapper_outer (reference run.py:159-170): outside debug mode a failed run logs
    {'errored': True} plus dataset_name, seed, method_name and domain_conf, in that order."""
    import run
    from insite_amd import config as C
    drv = C.driver_config()
    drv["setup"]["debug_mode"] = False
    r = run.run_one(drv, "EQ_4_A", "sindy", 3, 2.0, extra=["+backbone=no_such_backbone"])
    assert list(r) == ["errored", "dataset_name", "seed", "method_name", "domain_conf"]
    assert r["errored"] is True and r["seed"] == 3


def test_refine_terms_fold_matches_the_oracle():
    """ops.refine_terms (the product's per-coefficient arm masks) equals the oracle's coef_terms for per-arm,
    degree-4 and joint libraries."""
    from insite_amd import ops
    from insite_amd.library import polynomial_library
    from oracle import insite_refine_ref as Q
    for lib, A in ((polynomial_library(2, 2, True), 2), (polynomial_library(2, 4, False), 2),
                   (polynomial_library(1, 2, True), 4), (polynomial_library(2, 2, True, n_inputs=1), 1),
                   (polynomial_library(1, 2, True, n_inputs=2), 1)):
        mask, qexps, n_arms = ops.refine_terms(lib, A)
        c0 = np.ones((A, lib.n_terms))
        ref = Q.coef_terms(c0, lib.exps.astype(np.int64), lib.n_inputs)
        assert n_arms == Q.n_arms_of(c0, lib.n_inputs)
        assert mask.tolist() == [t[0] for t in ref]
        assert qexps[:, 0].tolist() == [t[1] for t in ref]
        assert [tuple(r) for r in qexps[:, 1:].tolist()] == [t[2] for t in ref]


@pytest.mark.parametrize("eq", ["EQ_4_B", "EQ_4_D"])
def test_pkpd_threefry_key_schedule_host_logic(monkeypatch, eq):
    """The host side of rng='threefry' (key threading, transforms, time grids, simulators) on CPU tensors,
    with the device word kernel stood in by the numpy restatement of jax's threefry_2x32 (test-only; the
    kernel itself is pinned in tests/test_gpu_threefry.py): the reference's cohorts come out."""
    from insite_amd import pkpd, threefry
    from oracle import jax_prng as J
    from oracle import ref_cohort as RC

    def words(key, n, device):
        w = J.threefry_2x32(np.array(key, np.uint32), np.arange(n, dtype=np.uint32)).astype(np.int64)
        return torch.from_numpy(w)

    monkeypatch.setattr(threefry, "_words", words)

    def rngs(kind, seed, subset, device):
        kp, ks = threefry.subset_streams(seed, "cpu")
        return pkpd._ThreefryRng(kp.key, "cpu"), pkpd._ThreefryRng(ks.key, "cpu")

    monkeypatch.setattr(pkpd, "subset_rngs", rngs)
    n = {"train": 30, "val": 5, "test": 4}
    c = pkpd.dataset_collection(eq, n, seed=1, max_seq_length=20, projection_horizon=3, device="cpu")
    ref = RC.make_collection(eq, n, seq_length=20, projection_horizon=3, seed=1)
    for mine, name in ((c.train_f, "train"), (c.val_f, "val"), (c.test_cf_one_step, "test_cf_one_step"),
                       (c.test_cf_treatment_seq, "test_cf_treatment_seq")):
        r = ref[name].data
        for k in ("sequence_lengths", "current_treatments", "active_entries"):
            assert np.array_equal(mine.data[k], r[k]), (name, k)
        for k in ("prev_outputs", "outputs", "static_features", "unscaled_outputs"):
            np.testing.assert_allclose(mine.data[k], r[k], rtol=0, atol=1e-11, err_msg=f"{name}/{k}")
