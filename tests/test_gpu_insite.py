"""GPU parity of the INSITE per-patient refinement (insite_refine_f64) against the
restatement oracle/insite_refine_ref.py (jax BFGS semantics; parity against jax itself is unpinned —
jax is absent — see that module).  Same algorithm in fp64 on both sides: statuses identical, refined
coefficients to 1e-7 relative (an ulp-level difference can move a line-search trial point; both stop at
the same gtol), predictions RMSE <= 1e-6 (north-star trajectory tolerance)."""
import numpy as np
import pytest
import torch

from oracle import insite_ref as R
from oracle import insite_refine_ref as Q

pytestmark = pytest.mark.gpu
EX = R.poly_library(3, 2, True)


@pytest.fixture(scope="module")
def model():
    coll = R.make_collection("EQ_4_C", {"train": 200, "val": 10, "test": 30}, seq_length=60, seed=2)
    tr = coll["train"]
    x, u, arm, rows = R.de_format(tr.data, tr.scaling_params)
    G, b = R.gram_moments(x, u, arm, rows, R.STANDARD_DT, EX)
    c0 = np.stack([R.stlsq_gram(G[a], b[a], 0.1, 0.5)[0] for a in range(2)])
    return coll, x, u, arm, c0


def _run(dev, V, arms, u, sl, c0, tau, lam=10.0):
    from insite_amd import ops
    from insite_amd.library import polynomial_library
    lib = polynomial_library(2, 2, True)
    preds, coef, status, iters = ops.insite_refine(torch.tensor(V, device=dev), torch.tensor(arms, device=dev),
                                                   torch.tensor(u, device=dev), torch.tensor(sl, device=dev), c0, lib,
                                                   R.STANDARD_DT, lam, tau)
    torch.cuda.synchronize()
    return preds.cpu().numpy(), coef.cpu().numpy(), status.cpu().numpy(), iters.cpu().numpy()


@pytest.mark.parametrize("tau", [1, 5])
def test_refine_matches_oracle(dev, model, tau):
    coll, x, u, arm, c0 = model
    rng = np.random.default_rng(tau)
    N, T = 150, x.shape[1]
    V = x[:N].copy()
    arms = np.repeat(arm[:N, None], T, axis=1).astype(np.int8)
    flip = rng.integers(10, T, N)
    for i in range(0, N, 3):                      # per-step treatment switches in a third of the rows
        arms[i, flip[i]:] = 1 - arms[i, flip[i]:]
    sl = rng.integers(1, T + 1, N).astype(np.int32)
    sl[:4] = [1, tau, tau + 1, T]
    preds, coef, status, iters = _run(dev, V, arms, u[:N], sl, c0, tau)
    for p in range(N):
        rp, rc, rs, ri = Q.refine_patient(V[p], arms[p], u[p], sl[p], c0, EX, R.STANDARD_DT, 10.0, tau)
        assert status[p] == rs, (p, status[p], rs)
        assert np.abs(coef[p] - rc).max() <= 1e-7 * max(1.0, np.abs(rc).max()), p
        assert np.sqrt(np.mean((preds[p] - rp) ** 2)) <= 1e-6
    assert (status[sl <= tau] == -1).all() and (iters[sl > tau] > 0).all()


def test_refine_matches_oracle_long_rows(dev):
    """T = 90 > 64: the refinement's per-step-load kernel (no window ring, no 64-bit arm mask) with the closed-form
    objective scans, against the oracle row by row (statuses, coefficients, predictions), arm switches included."""
    coll = R.make_collection("EQ_4_C", {"train": 120, "val": 10, "test": 10}, seq_length=90, seed=5)
    tr = coll["train"]
    x, u, arm, rows = R.de_format(tr.data, tr.scaling_params)
    G, b = R.gram_moments(x, u, arm, rows, R.STANDARD_DT, EX)
    c0 = np.stack([R.stlsq_gram(G[a], b[a], 0.1, 0.5)[0] for a in range(2)])
    rng = np.random.default_rng(90)
    N, T, tau = 100, x.shape[1], 5
    assert T > 64
    V = x[:N].copy()
    arms = np.repeat(arm[:N, None], T, axis=1).astype(np.int8)
    flip = rng.integers(10, T, N)
    for i in range(0, N, 2):
        arms[i, flip[i]:] = 1 - arms[i, flip[i]:]
    sl = rng.integers(1, T + 1, N).astype(np.int32)
    sl[:3] = [tau, tau + 1, T]
    preds, coef, status, iters = _run(dev, V, arms, u[:N], sl, c0, tau)
    for p in range(N):
        rp, rc, rs, ri = Q.refine_patient(V[p], arms[p], u[p], sl[p], c0, EX, R.STANDARD_DT, 10.0, tau)
        assert status[p] == rs, (p, status[p], rs)
        assert np.abs(coef[p] - rc).max() <= 1e-7 * max(1.0, np.abs(rc).max()), p
        assert np.sqrt(np.mean((preds[p] - rp) ** 2)) <= 1e-6


def test_refined_model_fits_better_than_global(dev, model):
    coll, x, u, arm, c0 = model
    N, T = 100, x.shape[1]
    arms = np.repeat(arm[:N, None], T, axis=1).astype(np.int8)
    sl = np.full(N, T, dtype=np.int32)
    preds, coef, status, _ = _run(dev, x[:N], arms, u[:N], sl, c0, 5)
    K = T - 5
    base = np.stack([Q.euler5_rollout(x[p, 0], arms[p], u[p], c0, EX, R.STANDARD_DT, T) for p in range(N)])
    e_ref = np.mean((x[:N, 1:K + 1] - preds[:, :K]) ** 2, axis=1)
    e_glob = np.mean((x[:N, 1:K + 1] - base[:, :K]) ** 2, axis=1)
    assert (e_ref <= e_glob * (1 + 1e-12)).all()
    assert (status == 0).mean() > 0.9


def test_plugin_insite_end_to_end(dev, model):
    """+backbone=insite: fit, refined one-step predictions (tau = 1, the reference's get_predictions
    default) and tau-step autoregressive predictions, against the oracle per row."""
    from insite_amd import config as C
    from insite_amd.sindy import SINDY
    coll, x, u, arm, c0 = model
    args = C.compose(["+backbone=insite", "+dataset=pkpd_sim", "dataset.equation_str=EQ_4_C",
                      "model.dataset_name=EQ_4_C", "model.sindy_threshold=0.1", "model.sindy_alpha=0.5",
                      "model.lam=10.0"])
    m = SINDY(args, device=dev)
    m.fit(coll["train"])
    assert m.insite and np.abs(m.joint_coefs - c0).max() < 1e-8
    m.joint_coefs = c0.copy()
    ds = coll["test_cf_one_step"]
    p = m.get_predictions(ds)
    assert p.shape == ds.data["outputs"].shape and not np.isnan(p).any()
    prev, stat = R.unscale_inputs(ds.data, ds.scaling_params)
    arms = np.argmax(ds.data["current_treatments"], axis=-1)
    sp = ds.scaling_params
    got = p[..., 0] * sp["output_stds"] + sp["output_means"]
    for i in range(0, prev.shape[0], 97):
        rp, *_ = Q.refine_patient(prev[i], arms[i], stat[i], int(ds.data["sequence_lengths"][i]), c0, EX,
                                  R.STANDARD_DT, 10.0, 1)
        assert np.sqrt(np.mean((got[i] - rp) ** 2)) <= 1e-6
    orig, allv, last = m.get_normalised_masked_rmse(ds, one_step_counterfactual=True)
    assert np.isfinite([orig, allv, last]).all()
    seq = coll["test_cf_treatment_seq"]
    ar = m.get_autoregressive_predictions(seq)
    assert ar.shape == (seq.data["outputs"].shape[0], m.projection_horizon, 1) and np.isfinite(ar).all()


def test_log_anchor_insite_vs_sindy_eq4a(dev):
    """Published accuracy anchors (results/2_main_table/final_with_insite.txt:126, :2346): one-step
    counterfactual RMSE "last" on EQ_4_A, 1000 train / 100 test patients — SINDy 0.1117 %, INSITE 0.0098 %.
    Our cohorts use a different RNG, so the check is the magnitude and the ~10x gain."""
    import run
    from insite_amd import config as C
    drv = C.driver_config()
    res = {}
    for method in ("sindy", "insite"):
        args = C.compose(C.run_overrides(drv, "EQ_4_A", method, 0, 2))
        res[method] = run.train_sindy_main(args, "EQ_4_A", device=dev)
    s, i = res["sindy"]["encoder_test_rmse_last"], res["insite"]["encoder_test_rmse_last"]
    assert 0.05 < s < 0.3 and i < 0.05 and i < s / 3, (s, i)
    assert res["insite"]["fine_tuned"] is True
    assert all(np.isfinite(res["insite"][f"decoder_test_rmse_{k}-step"]) for k in range(2, 7))


def _four_arm_problem(n_statics, n, seed):
    """A cancer_sim-like (n_statics = 1, F = 4) or EQ_5-like (n_statics = 2, F = 7) 4-arm cohort with
    per-step arm switches, and a global model off the planted one so the refinement has work to do."""
    from oracle import segments_ref as S
    rng = np.random.default_rng(seed)
    if n_statics == 1:
        coef = S.TRUE_COEF_U1
    else:
        coef = np.zeros((4, 7))
        coef[:, 1] = [0.2, -0.3, -0.25, 0.1]
        coef[:, 4] = [-0.4, 0.0, -0.6, -0.2]
        coef[1:, 5] = [0.3, -0.2, 0.25]
        coef[::2, 0] = [0.05, -0.05]
    x, u, arm, _ = S.synthetic_cohort(n, 60, rng, switch_p=0.1, noise=0.01, dt=1 / 6, coef=coef,
                                      n_statics=n_statics)
    c0 = coef * (1.0 + rng.normal(0.0, 0.1, size=coef.shape))
    c0[np.abs(coef) == 0] = 0.0
    c0[0, -1] = 5e-4                              # below the 1e-3 mask: never refined, kept as is
    return x[:, :60].copy(), u, arm.astype(np.int8), c0, R.poly_library(1 + n_statics, 2, True)


@pytest.mark.parametrize("n_statics,tau", [(1, 1), (1, 5), (2, 5)])
def test_refine_four_arms_matches_oracle(dev, n_statics, tau):
    """insite_refine_arms_f64 (int8 arms, NA = 4; sindy.py:484-550) against the oracle per row:
    cancer_sim (4 x 4 model, 6 active) and EQ_5-like (4 x 7 model, 12 active: the M = 16 kernel)."""
    from insite_amd import ops
    from insite_amd.library import polynomial_library
    V, u, arms, c0, ex = _four_arm_problem(n_statics, 48, 3 + n_statics)
    N, T = V.shape
    rng = np.random.default_rng(tau)
    sl = rng.integers(1, T + 1, N).astype(np.int32)
    sl[:3] = [tau, tau + 1, T]
    lib = polynomial_library(n_statics, 2, True)
    preds, coef, status, iters = ops.insite_refine(torch.tensor(V, device=dev), torch.tensor(arms, device=dev),
                                                   torch.tensor(u, device=dev), torch.tensor(sl, device=dev), c0, lib,
                                                   1 / 6, 10.0, tau)
    torch.cuda.synchronize()
    preds, coef, status = preds.cpu().numpy(), coef.cpu().numpy(), status.cpu().numpy()
    for p in range(N):
        rp, rc, rs, _ = Q.refine_patient(V[p], arms[p], u[p], sl[p], c0, ex, 1 / 6, 10.0, tau)
        assert status[p] == rs, (p, status[p], rs)
        assert np.abs(coef[p] - rc).max() <= 1e-7 * max(1.0, np.abs(rc).max()), p
        assert np.sqrt(np.mean((preds[p] - rp) ** 2)) <= 1e-6
    assert (coef[:, 0, -1] == c0[0, -1]).all()
    assert (status[sl <= tau] == -1).all() and (status[sl > tau] == 0).mean() > 0.8


@pytest.mark.parametrize("n_arms", [2, 4])
def test_refine_dense_model_matches_oracle(dev, n_arms):
    """A dense global model (every coefficient above the 1e-3 mask: 14 or 28 active, the latter past the
    16-coefficient register kernel) is refined, not rejected: the M = 36 scratch-resident instantiation
    runs the same BFGS arithmetic as the oracle."""
    from insite_amd import ops
    from insite_amd.library import polynomial_library
    V, u, arms, c0, ex = _four_arm_problem(2, 40, 11)
    tau = 5
    if n_arms == 2:
        arms = (arms % 2).astype(np.int8)
    c0 = c0[:n_arms].copy()
    c0[np.abs(c0) <= 1e-3] = 0.02                  # every term active
    N, T = V.shape
    sl = np.full(N, T, dtype=np.int32)
    sl[:2] = [tau, tau + 1]
    lib = polynomial_library(2, 2, True)
    preds, coef, status, iters = ops.insite_refine(torch.tensor(V, device=dev), torch.tensor(arms, device=dev),
                                                   torch.tensor(u, device=dev),
                                                   torch.tensor(sl, device=dev), c0, lib, 1 / 6, 10.0, tau)
    torch.cuda.synchronize()
    preds, coef, status = preds.cpu().numpy(), coef.cpu().numpy(), status.cpu().numpy()
    assert coef.shape == (N, n_arms, 7)
    for p in range(N):
        rp, rc, rs, _ = Q.refine_patient(V[p], arms[p], u[p], sl[p], c0, ex, 1 / 6, 10.0, tau)
        assert status[p] == rs, (p, status[p], rs)
        assert np.abs(coef[p] - rc).max() <= 1e-7 * max(1.0, np.abs(rc).max()), p
        assert np.sqrt(np.mean((preds[p] - rp) ** 2)) <= 1e-6
    assert status[0] == -1 and (status[1:] >= 0).all()


@pytest.mark.parametrize("name,n_statics", [("cancer_sim", 1), ("EQ_5_B", 2)])
def test_plugin_insite_four_arms(dev, name, n_statics):
    """+backbone=insite on a 4-arm dataset: segment discovery, then per-row refinement; the EQ_5
    refinement binds u1 to static_features[0] as the reference does (sindy.py:536)."""
    from insite_amd.sindy import SINDY
    from test_gpu_segments import _Subset
    V, u, arms, c0, ex = _four_arm_problem(n_statics, 300, 7)
    N, T = V.shape
    x = np.concatenate([V, V[:, -1:]], axis=1)          # [N, T + 1]: prev_outputs = V
    sl = np.full(N, T, dtype=np.int64)
    sl[::4] = 3
    args = {"model": {"dataset_name": name, "dim_treatments": 4, "dim_static_features": n_statics,
                      "dim_outcomes": 1, "sindy_threshold": 0.001, "sindy_alpha": 0.5, "insite": True,
                      "lam": 10.0},
            "dataset": {"projection_horizon": 5}, "exp": {"unscale_rmse": True, "percentage_rmse": True}}
    m = SINDY(args, device=dev)
    ds = _Subset(x, u, arms, sl)
    m.fit(ds)
    assert m.joint_coefs.shape == (4, ex.shape[0])
    m.joint_coefs = c0.copy()                          # a global model with <= 16 active coefficients
    p = m.get_predictions(ds)[..., 0]
    uq = u.copy()
    if n_statics == 2:
        uq[:, 1] = uq[:, 0]
    for i in range(0, N, 23):
        rp, *_ = Q.refine_patient(V[i], arms[i], uq[i], int(sl[i]), c0, ex, m.dt, 10.0, 1)
        assert np.sqrt(np.mean((p[i] - rp) ** 2)) <= 1e-6, i


@pytest.mark.parametrize("n_arms", [2, 4])
def test_refine_binned_rows_bitwise_equal_identity_order(dev, n_arms):
    """Rows binned by seq_len (ABI 4 row_order, the default) are scheduling only: preds, coefficients,
    statuses and iteration counts are bitwise those of the identity lane order (ragged seq_len, incl.
    rows <= tau that are skipped)."""
    from insite_amd import ops, cohort
    from insite_amd.library import polynomial_library
    N, T, tau = 20_000, 60, 5
    coh = cohort.synthetic_pkpd(N, T, seed=4, device=dev, equation="EQ_4_C")
    V = coh.x[:, :T].contiguous()
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    flip = torch.randint(1, T, (N, 1), generator=g, device=dev)
    base = coh.arm[:, None].to(torch.int64)
    if n_arms == 4:
        base = torch.randint(0, 4, (N, 1), generator=g, device=dev)
    arm = torch.where(torch.arange(T, device=dev)[None, :] >= flip, (base + 1) % n_arms, base).to(torch.int8)
    sl = torch.randint(1, T + 1, (N,), generator=g, device=dev, dtype=torch.int32)
    lib = polynomial_library(2, 2, True)
    c0 = np.zeros((n_arms, lib.n_terms))
    c0[:, 4] = -1.1
    c0[1, 1], c0[1, 5] = -0.145, -1.02
    outs = [ops.insite_refine(V, arm.contiguous(), coh.u, sl, c0, lib, 10.0 / T, 10.0, tau, binned=b)
            for b in (True, False)]
    torch.cuda.synchronize()
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert (outs[0][2][sl <= tau] == -1).all() and (outs[0][2][sl > tau] >= 0).all()


@pytest.mark.parametrize("N,T", [(1, 7), (63, 60), (100, 60), (4097, 33)])
def test_refine_prepare_layout_equals_torch(dev, N, T):
    """insite_refine_prepare_f64 (ABI 7): one device pass from the reference's patient-major V / per-step arms to
    the refinement's time-major V and bit-packed (or int8) arms, bitwise what the torch transposes and
    ops.pack_arm_bits give, ragged N (partial words and waves) included; 2-valued arms for the bit mask."""
    from insite_amd import ops
    g = torch.Generator(device=dev)
    g.manual_seed(N + T)
    V = torch.randn((N, T), generator=g, device=dev, dtype=torch.float64)
    arm2 = torch.randint(0, 2, (N, T), generator=g, device=dev, dtype=torch.int8)
    Vt, bits = ops.refine_prepare(V, arm2, bits=True)
    assert torch.equal(Vt, V.t().contiguous())
    assert torch.equal(bits, ops.pack_arm_bits(arm2.t().contiguous(), N))
    arm4 = torch.randint(0, 4, (N, T), generator=g, device=dev, dtype=torch.int8)
    Vt4, a8 = ops.refine_prepare(V, arm4, bits=False)
    assert torch.equal(Vt4, Vt) and torch.equal(a8, arm4.t().contiguous())
    with pytest.raises(ValueError):
        ops.refine_prepare(V, arm4 + 2, bits=True)


@pytest.mark.parametrize("N,T", [(5, 7), (100, 60), (4097, 33)])
def test_refine_prepare_finish_with_row_order(dev, N, T):
    """Binned layout (ABI 7): insite_refine_prepare_f64 with a row order gathers row order[l] into column l, and
    insite_refine_finish_f64 scatters time-major columns back to patient-major rows -- bitwise torch indexing."""
    from insite_amd import ops
    g = torch.Generator(device=dev)
    g.manual_seed(7 * N + T)
    V = torch.randn((N, T), generator=g, device=dev, dtype=torch.float64)
    arm = torch.randint(0, 2, (N, T), generator=g, device=dev, dtype=torch.int8)
    order = torch.randperm(N, generator=g, device=dev).to(torch.int32)
    Vt, bits = ops.refine_prepare(V, arm, bits=True, order=order)
    idx = order.long()
    assert torch.equal(Vt, V[idx].t().contiguous())
    assert torch.equal(bits, ops.pack_arm_bits(arm[idx].t().contiguous(), N))
    back = ops.refine_finish(Vt, order, N)
    assert torch.equal(back, V)
    assert torch.equal(ops.refine_finish(V.t().contiguous(), None, N), V)
    # ABI 8: the same passes move the per-row side arrays (statics, sequence lengths in; coefficients, statuses,
    # iteration counts out)
    u = torch.randn((N, 2), generator=g, device=dev, dtype=torch.float64)
    sl = torch.randint(0, T, (N,), generator=g, device=dev, dtype=torch.int32)
    Vt2, bits2, u_l, sl_l = ops.refine_prepare(V, arm, bits=True, order=order, u=u, seq_len=sl)
    assert torch.equal(Vt2, Vt) and torch.equal(bits2, bits)
    assert torch.equal(u_l, u[idx]) and torch.equal(sl_l, sl[idx])
    c_l = torch.randn((N, 2, 7), generator=g, device=dev, dtype=torch.float64)
    s_l = torch.randint(-1, 4, (N,), generator=g, device=dev, dtype=torch.int32)
    i_l = torch.randint(0, 9, (N,), generator=g, device=dev, dtype=torch.int32)
    P, c, s_, it = ops.refine_finish(Vt, order, N, lane_outputs=(c_l, s_l, i_l))
    assert torch.equal(P, V)
    for got, lane in ((c, c_l), (s_, s_l), (it, i_l)):
        want = torch.empty_like(lane).index_copy_(0, idx, lane)
        assert torch.equal(got, want)


def test_insite_refine_plan_equals_eager(dev):
    """ops.plan_insite_refine (the INSITE bench step: sort, gather, kernel, scatter -- 4 C calls, no host sync)
    returns bitwise what ops.insite_refine(binned=True) returns, over repeated calls."""
    from insite_amd import cohort, ops
    N, T = 20_000, 60
    coh = cohort.synthetic_pkpd(N, T, seed=31, device=dev, equation="EQ_4_C")
    V = coh.x[:, :T].contiguous()
    g = torch.Generator(device=dev)
    g.manual_seed(32)
    flip = torch.randint(1, T, (N, 1), generator=g, device=dev)
    arm = torch.where(torch.arange(T, device=dev)[None, :] >= flip, 1 - coh.arm[:, None].to(torch.int64),
                      coh.arm[:, None].to(torch.int64)).to(torch.int8).contiguous()
    sl = torch.randint(1, T, (N,), generator=g, device=dev, dtype=torch.int32)
    c0 = np.zeros((2, coh.lib.n_terms))
    c0[0, 4], c0[1, 1], c0[1, 5] = -1.1107592869834308, -0.14540553723951796, -1.0234639833519243
    plan = ops.plan_insite_refine(V, arm, coh.u, sl, c0, coh.lib, 10.0 / T, 10.0, 5)
    want = ops.insite_refine(V, arm, coh.u, sl, c0, coh.lib, 10.0 / T, 10.0, 5, binned=True)
    for _ in range(2):
        got = plan()
        torch.cuda.synchronize()
        for a, b in zip(got, want):
            assert torch.equal(a, b)


@pytest.mark.parametrize("N,T", [(5_000, 60), (4_097, 33), (130, 64), (777, 7)])
def test_windowed_refine_equals_per_step_loads(dev, N, T):
    """The windowed M <= 4 kernels (LDS ring of observation slots filled by LDS-DMA, arm masks in registers,
    wave-uniform flat BFGS loop; identity lane order) against the per-step-load kernels (selected here by passing an
    explicit identity row order): predictions, coefficients, statuses, iteration and evaluation counts bitwise equal,
    incl. a partial last wave (inert lanes), odd N (padded even leading dimension) and short T."""
    from insite_amd import cohort, ops
    coh = cohort.synthetic_pkpd(N, T, seed=N + T, device=dev, equation="EQ_4_C")
    V = coh.x[:, :T].contiguous()
    g = torch.Generator(device=dev)
    g.manual_seed(N * 3 + T)
    flip = torch.randint(1, max(2, T), (N, 1), generator=g, device=dev)
    arm = torch.where(torch.arange(T, device=dev)[None, :] >= flip, 1 - coh.arm[:, None].to(torch.int64),
                      coh.arm[:, None].to(torch.int64)).to(torch.int8).contiguous()
    sl = torch.randint(1, T + 1, (N,), generator=g, device=dev, dtype=torch.int32)
    c0 = np.zeros((2, coh.lib.n_terms))
    c0[0, 4], c0[1, 1], c0[1, 5] = -1.1107592869834308, -0.14540553723951796, -1.0234639833519243
    Vt, bits = ops.refine_prepare(V, arm, bits=True)
    assert Vt.stride(0) % 2 == 0
    ident = torch.arange(N, device=dev, dtype=torch.int32)
    nf_w = torch.empty((N,), dtype=torch.int32, device=dev)
    nf_l = torch.empty((N,), dtype=torch.int32, device=dev)
    w = ops.insite_refine_tm(Vt, bits, coh.u, sl, c0, coh.lib, 10.0 / T, 10.0, 5, nfev=nf_w)
    l_ = ops.insite_refine_tm(Vt, bits, coh.u, sl, c0, coh.lib, 10.0 / T, 10.0, 5, order=ident, nfev=nf_l)
    torch.cuda.synchronize()
    for a, b in zip(w, l_):
        assert torch.equal(a, b)
    assert torch.equal(nf_w, nf_l)


@pytest.mark.parametrize("N,T,ld,m", [(5_000, 60, 60, 3), (4_097, 34, 34, 3), (130, 64, 64, 2), (777, 7, 8, 3),
                                      (1, 2, 2, 3), (65, 33, 40, 2)])
def test_refine_rows_layout_equals_prepare_route(dev, N, T, ld, m):
    """insite_refine_rows_f64 (ABI 9: the windowed kernel on the patient-major rows gathered through the lane order,
    predictions stored through the LDS ring as row segments, no prepare / finish passes) against the prepare /
    kernel / finish route: predictions, coefficients, statuses, iteration and evaluation counts bitwise equal.  Ragged
    seq_len (rows <= tau skipped), a partial last wave, padded leading dimensions, T = 2 and the M = 2 / M = 3
    kernels; binned and identity lane orders; the plan takes the same route."""
    from insite_amd import cohort, ops
    coh = cohort.synthetic_pkpd(N, T, seed=N + 7 * T, device=dev, equation="EQ_4_C")
    V = torch.zeros((N, ld), dtype=torch.float64, device=dev)[:, :T]
    V.copy_(coh.x[:, :T])
    g = torch.Generator(device=dev)
    g.manual_seed(N * 5 + T)
    flip = torch.randint(1, max(2, T), (N, 1), generator=g, device=dev)
    arm = torch.zeros((N, ld), dtype=torch.int8, device=dev)[:, :T]
    arm.copy_(torch.where(torch.arange(T, device=dev)[None, :] >= flip, 1 - coh.arm[:, None].to(torch.int64),
                          coh.arm[:, None].to(torch.int64)).to(torch.int8))
    sl = torch.randint(1, T + 1, (N,), generator=g, device=dev, dtype=torch.int32)
    c0 = np.zeros((2, coh.lib.n_terms))
    c0[0, 4], c0[1, 1] = -1.1107592869834308, -0.14540553723951796
    if m == 3:
        c0[1, 5] = -1.0234639833519243
    Vc, ac = V.contiguous(), arm.contiguous()
    for binned in (True, False):
        nf_r = torch.empty((N,), dtype=torch.int32, device=dev)
        nf_p = torch.empty((N,), dtype=torch.int32, device=dev)
        r = ops.insite_refine(V, arm, coh.u, sl, c0, coh.lib, 10.0 / T, 10.0, 5, binned=binned, nfev=nf_r, rows=True)
        p = ops.insite_refine(Vc, ac, coh.u, sl, c0, coh.lib, 10.0 / T, 10.0, 5, binned=binned, nfev=nf_p, rows=False)
        torch.cuda.synchronize()
        for a, b in zip(r, p):
            assert torch.equal(a, b)
        assert torch.equal(nf_r, nf_p)
        assert (r[2][sl <= 5] == -1).all()
    plan = ops.plan_insite_refine(V, arm, coh.u, sl, c0, coh.lib, 10.0 / T, 10.0, 5)
    assert plan.mode == "rows"
    got = plan()
    torch.cuda.synchronize()
    for a, b in zip(got, p):
        assert torch.equal(a, b)
    # lanes binned by window and the previous call's evaluation counts (the insite line's default order): the first
    # call bins on zero counts, the next ones on the counts the previous call wrote -- every call's outputs bitwise
    # those of the seq_len order, the counts those of the eager route
    nplan = ops.plan_insite_refine(V, arm, coh.u, sl, c0, coh.lib, 10.0 / T, 10.0, 5, order="nfev")
    assert nplan.mode == "rows" and nplan.kernel_call == 2
    for _ in range(3):
        got = nplan()
        torch.cuda.synchronize()
        for a, b in zip(got, p):
            assert torch.equal(a, b)
        assert torch.equal(nplan.nfev, nf_p)
        assert torch.equal(torch.sort(nplan.order).values, torch.arange(N, device=dev, dtype=torch.int32))


def test_refine_rows_unsupported_shapes_fall_back(dev):
    """Outside the windowed row kernel's shape (odd leading dimension, T > 64, four arms) the library answers
    INSITE_E_UNSUPPORTED without launching, insite_refine(rows=None) takes the prepare route and rows=True raises."""
    from insite_amd import cohort, ops
    for N, T in ((300, 33), (300, 70)):
        coh = cohort.synthetic_pkpd(N, T, seed=3, device=dev, equation="EQ_4_C")
        V = coh.x[:, :T].contiguous()
        arm = coh.arm[:, None].expand(N, T).to(torch.int8).contiguous()
        sl = torch.full((N,), T, dtype=torch.int32, device=dev)
        c0 = np.zeros((2, coh.lib.n_terms))
        c0[0, 4], c0[1, 1] = -1.1, -0.145
        a = ops.insite_refine(V, arm, coh.u, sl, c0, coh.lib, 10.0 / T, 10.0, 5)
        b = ops.insite_refine(V, arm, coh.u, sl, c0, coh.lib, 10.0 / T, 10.0, 5, rows=False)
        torch.cuda.synchronize()
        for x, y in zip(a, b):
            assert torch.equal(x, y)
        with pytest.raises(ValueError):
            ops.insite_refine(V, arm, coh.u, sl, c0, coh.lib, 10.0 / T, 10.0, 5, rows=True)
        assert ops.plan_insite_refine(V, arm, coh.u, sl, c0, coh.lib, 10.0 / T, 10.0, 5).mode == "prepare"


def test_plugin_insite_rejects_non_finite_refined_predictions(dev, model, monkeypatch):
    """The reference asserts that the refined predictions hold no NaN or Inf (sindy.py:710); the plugin raises the
    same AssertionError when the refinement returns a row whose refined model blew up."""
    from insite_amd import config as C
    from insite_amd import sindy as S
    coll, x, u, arm, c0 = model
    args = C.compose(["+backbone=insite", "+dataset=pkpd_sim", "dataset.equation_str=EQ_4_C",
                      "model.dataset_name=EQ_4_C", "model.sindy_threshold=0.1", "model.sindy_alpha=0.5",
                      "model.lam=10.0"])
    m = S.SINDY(args, device=dev)
    m.fit(coll["train"])
    real = S.ops.insite_refine

    def blown(*a, **k):
        preds, coef, status, iters = real(*a, **k)
        preds[3, -1] = float("inf")
        return preds, coef, status, iters

    monkeypatch.setattr(S.ops, "insite_refine", blown)
    with pytest.raises(AssertionError, match="NaN or Inf"):
        m.get_predictions(coll["test_cf_one_step"])


@pytest.mark.parametrize("N,T,m,refill,blocks", [(20_000, 60, 3, None, None), (5_000, 60, 2, "1", None),
                                                 (777, 34, 3, "64", "2"), (130, 8, 3, "8", "1"),
                                                 (3_000, 60, 3, "8", "2")])
def test_refine_rows_dynamic_assignment_equals_static(dev, monkeypatch, N, T, m, refill, blocks):
    """insite_refine_rows_f64's dynamic lane -> row assignment (a wave's idle lanes take the next rows from a
    device-wide queue head with one atomic once at least `refill` of them are idle, INSITE_REFINE_DYN_REFILL; the
    final scan in its own kernel from the written coefficients) against the static one-row-per-lane kernel
    (INSITE_REFINE_DYN=0): every output bitwise equal, incl. rows <= tau (finished at claim), thresholds 1 / 8 / 64
    and a persistent grid of 1 or 2 blocks (INSITE_REFINE_DYN_BLOCKS: every lane cycles through many rows)."""
    from insite_amd import cohort, ops
    coh = cohort.synthetic_pkpd(N, T, seed=N + 3 * T, device=dev, equation="EQ_4_C")
    V = coh.x[:, :T].contiguous()
    g = torch.Generator(device=dev)
    g.manual_seed(N + T)
    flip = torch.randint(1, max(2, T), (N, 1), generator=g, device=dev)
    arm = torch.where(torch.arange(T, device=dev)[None, :] >= flip, 1 - coh.arm[:, None].to(torch.int64),
                      coh.arm[:, None].to(torch.int64)).to(torch.int8).contiguous()
    sl = torch.randint(1, T + 1, (N,), generator=g, device=dev, dtype=torch.int32)
    c0 = np.zeros((2, coh.lib.n_terms))
    c0[0, 4], c0[1, 1] = -1.1107592869834308, -0.14540553723951796
    if m == 3:
        c0[1, 5] = -1.0234639833519243
    if refill is not None:
        monkeypatch.setenv("INSITE_REFINE_DYN_REFILL", refill)
    if blocks is not None:
        monkeypatch.setenv("INSITE_REFINE_DYN_BLOCKS", blocks)
    outs = {}
    for dyn in ("1", "0"):
        monkeypatch.setenv("INSITE_REFINE_DYN", dyn)
        nf = torch.empty((N,), dtype=torch.int32, device=dev)
        r = ops.insite_refine(V, arm, coh.u, sl, c0, coh.lib, 10.0 / T, 10.0, 5, nfev=nf, rows=True)
        torch.cuda.synchronize()
        outs[dyn] = tuple(t.clone() for t in r) + (nf,)
    for a, b in zip(outs["1"], outs["0"]):
        assert torch.equal(a, b)


F4_COEF = [[0.0, 0.20, 0.0, 0.0], [0.0, 0.0, 0.0, -0.60], [0.0, -0.30, 0.0, 0.0], [0.0, -0.25, 0.0, -0.90]]


@pytest.mark.parametrize("N,joint,T", [(3_000, False, 60), (517, False, 60), (2_000, True, 60), (600, False, 80)])
def test_cooperative_dense_refine_equals_single_lane(dev, monkeypatch, N, joint, T):
    """The cooperative kernel for the dense 4-arm models (8 lanes per row, H rows and coordinates distributed,
    INSITE_REFINE_COOP) against the one-row-per-lane M = 16 kernel (INSITE_REFINE_COOP=0): predictions,
    coefficients, statuses, iteration and evaluation counts bitwise equal (every sum over coefficients is taken in the
    single-lane kernel's order and without contraction in both, insite_refine.hip "NC") -- the dense per-arm model
    (16 active coefficients, cancer_sim's shape) and the joint one-ODE model over (x, chemo, radio, u0); ragged
    seq_len incl. rows <= tau, a partial last wave; T = 80 takes the kernel's unstaged path (rows read per step,
    T > 64)."""
    from insite_amd import cohort, ops
    from insite_amd.library import polynomial_library
    coh = cohort.synthetic_segments(N, T, seed=N + 11, device=dev, coef=F4_COEF, dt=0.1)
    V = coh.x[:T, :N].t().contiguous()
    arm = coh.arm[:, :N].t().contiguous()
    g = torch.Generator(device=dev)
    g.manual_seed(N)
    sl = torch.randint(1, T + 1, (N,), generator=g, device=dev, dtype=torch.int32)
    if joint:
        lib = polynomial_library(1, 2, True, n_inputs=2)
        c0 = np.array([[-0.36, 0.33, 0.49, 0.074, 0.80, -0.45, -0.45, -0.29, 0.19, -1.15, -0.34]])
    else:
        lib = coh.lib
        base = np.array(F4_COEF) * 1.1
        c0 = np.where(base != 0, base, 0.01)
    outs = {}
    for coop in ("1", "0"):
        monkeypatch.setenv("INSITE_REFINE_COOP", coop)
        nf = torch.empty((N,), dtype=torch.int32, device=dev)
        r = ops.insite_refine(V, arm, coh.u, sl, c0, lib, coh.dt, 10.0, 5, nfev=nf)
        torch.cuda.synchronize()
        outs[coop] = tuple(t.clone() for t in r) + (nf,)
    assert (outs["1"][2][sl <= 5] == -1).all() and (outs["1"][2][sl > 5] >= 0).all()
    for a, b in zip(outs["1"], outs["0"]):
        assert torch.equal(a, b)
    # the cooperative kernel on the reference's own rows (insite_refine_rows_f64 with 4 arms, T <= 64) against its
    # prepare / kernel / finish route, and the 4-arm line's plan with its lanes binned by window and the previous
    # call's evaluation counts: three consecutive calls, outputs and row-order counts bitwise those of the eager route
    monkeypatch.setenv("INSITE_REFINE_COOP", "1")
    nf_p = torch.empty((N,), dtype=torch.int32, device=dev)
    rp = ops.insite_refine(V, arm, coh.u, sl, c0, lib, coh.dt, 10.0, 5, nfev=nf_p, rows=False)
    torch.cuda.synchronize()
    for a, b in zip(rp + (nf_p,), outs["1"]):
        assert torch.equal(a, b)
    nplan = ops.plan_insite_refine(V, arm, coh.u, sl, c0, lib, coh.dt, 10.0, 5, order="nfev")
    assert (nplan.mode, nplan.kernel_call) == (("rows", 2) if T <= 64 else ("prepare", 3))
    for _ in range(3):
        got = nplan()
        torch.cuda.synchronize()
        for a, b in zip(got, outs["1"][:4]):
            assert torch.equal(a, b)
        assert torch.equal(nplan.nfev, outs["1"][4])


def test_refine_rows_on_bench_cohort_sampled_against_oracle(dev):
    """the INSITE line's OWN 1M-row cohort (bench.insite_rows, seed as ``bench.py --config
    insite``) through the product call the line times (ops.plan_insite_refine: the device seq_len sort +
    insite_refine_rows_f64 on binned lanes), ~4k sampled rows -- the first and last 64 lanes of the binned order
    among them -- against oracle/insite_refine_ref.refine_patient (bench.insite_parity, the line's own parity
    check): refined coefficients to 1e-7 and prediction RMSE <= 1e-6 on EVERY sampled row; statuses and iteration
    counts equal on >= 99.5 % of them.  The rest (7 of 4,349 on the first box run, 0.16 %) are rows where the two
    roundings of the objective -- the kernel's closed-form scans (INSITE_REFINE_CF) and the oracle's sub-step form --
    end the search differently at rounding-level flatness (e.g. converged vs a failed final zoom) with the SAME
    iterate: their coefficients still agree to ~1e-10."""
    import bench
    from insite_amd import ops
    coh, V, arm, sl, c0, dt = bench.insite_rows(1_000_000, 60, 1, dev)
    plan = ops.plan_insite_refine(V, arm, coh.u, sl, c0, coh.lib, dt, 10.0, 5)
    preds, coef, status, iters = plan()
    torch.cuda.synchronize()
    o = plan.order.long()
    par = bench.insite_parity(V, arm, coh.u, sl, c0, coh.lib, dt, 10.0, 5, preds, coef, status, iters,
                              extra=(o[:64].cpu().numpy(), o[-64:].cpu().numpy()))
    print(par)
    assert par["rows_sampled"] >= 4096
    assert par["status_equal_frac"] >= 0.995 and par["iterations_equal_frac"] >= 0.995, par
    assert par["coef_linf"] <= 1e-7, par
    assert par["pred_rmse"] <= 1e-6, par


def test_refine_rows_revert_mode_on_bench_cohort_sampled_against_oracle(dev):
    """the literal status-3 revert of sindy.py:628-631 (``insite_revert_on_zoom_fail: true``) at the
    INSITE line's bench size -- the line's own 1M-row cohort through the product call with the revert flag, ~4k sampled
    rows against oracle/insite_refine_ref.refine_patient(revert_on_zoom_fail=True).  On every row whose status agrees
    the predictions agree to the default mode's bar (RMSE <= 1e-6) and so do the coefficients; statuses agree on >= 99.5
    % of the rows; on the few status-mismatch rows (the closed-form scans' rounding ending a search as converged where
    the oracle's sub-step form ends it in a failed zoom, or the reverse) the side that reports status 3 holds exactly
    c0 -- the difference there is the revert decision itself, not the refinement."""
    import bench
    from insite_amd import ops
    coh, V, arm, sl, c0, dt = bench.insite_rows(1_000_000, 60, 1, dev)
    plan = ops.plan_insite_refine(V, arm, coh.u, sl, c0, coh.lib, dt, 10.0, 5, revert_on_zoom_fail=True)
    preds, coef, status, iters = plan()
    torch.cuda.synchronize()
    o = plan.order.long()
    par = bench.insite_parity(V, arm, coh.u, sl, c0, coh.lib, dt, 10.0, 5, preds, coef, status, iters,
                              extra=(o[:64].cpu().numpy(), o[-64:].cpu().numpy()), revert=True)
    print(par)
    assert par["rows_sampled"] >= 4096
    assert par["status_equal_frac"] >= 0.995, par
    assert par["coef_linf_status_equal"] <= 1e-7, par
    assert par["pred_rmse_status_equal"] <= 1e-6, par
    assert par["mismatch_reverted_side_is_c0"], par
    # statuses 3 on the GPU side keep c0 exactly over the whole cohort
    s3 = (status == 3).nonzero().flatten()
    if s3.numel():
        c0t = torch.as_tensor(np.asarray(c0, dtype=np.float64), device=dev)
        assert torch.equal(coef.index_select(0, s3), c0t.expand(s3.numel(), *c0t.shape))
