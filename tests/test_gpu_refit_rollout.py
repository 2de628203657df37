"""C4's per-patient refit folded into its rollout (insite_refit_rollout_moments_f64, ABI 5): each lane refits
its factual arm's row from its moments in the rollout prologue (closed-form ridge iterations on the rank-2
Gram) instead of a separate patient_fit_kernel launch plus an HBM round trip of the coefficient rows.

* against the two-call path (fit_per_patient_moments + the per-row rollout): y bitwise, refits bitwise,
  same supports and iteration counts -- both run the same patient_refit arithmetic;
* against the oracle: R.per_patient_fit (row-form STLSQ from the global support, the reference's
  LSQIntialMask per patient, pkpd_simulation.py:791-800) and R.rollout with those per-patient coefficients
  (predict_with_reduced_coefs, sindy.py:767-778): coefficients L-inf < 1e-8, supports and iteration counts
  equal, y rtol 1e-10 -- on the golden EQ_4_A/C cohorts and a sample of the C4 bench's 1M x 60 cohort;
* edge cases: ragged rows (< 5 rows keep the global model), a partial last tile, alpha = 0 refused.
"""
import numpy as np
import pytest
import torch

from oracle import insite_ref as R

pytestmark = pytest.mark.gpu


def _two_call(ops, mom, u, arm, rows, T_fit, lib, coef, y0, bits, dt, T):
    pc, pm, pi = ops.fit_per_patient_moments(mom, u, arm, rows, T_fit, lib, coef, 0.1, 0.5)
    y = ops.rollout(y0, u, bits, pc, lib, dt, method="euler5", T=T, layout="time_bits")
    return pc, pm, pi, y


@pytest.mark.parametrize("N,T,ragged", [(100_000, 60, False), (3_001, 60, True), (777, 37, True)])
def test_fold_matches_two_call_path_bitwise(dev, N, T, ragged):
    from insite_amd import cohort, ops
    coh = cohort.synthetic_pkpd(N, T, seed=11, device=dev, equation="EQ_4_C", layout="time")
    rows = coh.rows
    if ragged:
        g = torch.Generator(device=dev)
        g.manual_seed(N)
        rows = torch.randint(0, T - 1, (N,), generator=g, device=dev, dtype=torch.int32)
    lib = coh.lib
    coef, _, _, _, _, mom = ops.gram_moments(coh.x, coh.u, coh.arm, rows, coh.dt, lib, 0.1, 0.5, layout="time")
    bits = cohort.counterfactual_arms(coh.arm, T, seed=13, layout="time_bits")
    pc, pm, pi, y2 = _two_call(ops, mom, coh.u, coh.arm, rows, T, lib, coef, coh.y0, bits, coh.dt, T)
    fc = torch.empty_like(pc)
    fm = torch.empty_like(pm)
    fi = torch.empty_like(pi)
    y = ops.refit_rollout_moments(mom, coh.u, coh.arm, rows, T, lib, coef, 0.1, 0.5, coh.y0, bits, coh.dt, T,
                                  fits=(fc, fm, fi))
    y_only = ops.refit_rollout_moments(mom, coh.u, coh.arm, rows, T, lib, coef, 0.1, 0.5, coh.y0, bits, coh.dt, T)
    torch.cuda.synchronize()
    assert torch.equal(y, y2) and torch.equal(y_only, y2)
    assert torch.equal(fc, pc) and torch.equal(fm, pm) and torch.equal(fi, pi)
    if ragged:
        short = (rows < 5).nonzero().flatten()
        assert short.numel() > 0 and (pi[short] == 0).all()


@pytest.mark.parametrize("eq", ["EQ_4_A", "EQ_4_C"])
def test_fold_matches_oracle_on_golden(dev, eq):
    import os
    from insite_amd import ops, cohort
    from insite_amd.library import polynomial_library
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", f"discovery_{eq.lower()}.npz"))
    lib = polynomial_library(2, 2, True)
    exps = lib.exps.astype(np.int64)
    dt = float(g["dt"])
    N, T = g["x"].shape
    x = torch.tensor(np.ascontiguousarray(g["x"].T), device=dev)
    u = torch.tensor(g["u"], device=dev)
    arm = torch.tensor(g["arm"], device=dev, dtype=torch.int8)
    rows = torch.tensor(g["rows"], device=dev, dtype=torch.int32)
    coef, _, _, _, _, mom = ops.gram_moments(x, u, arm, rows, dt, lib, 0.1, 0.5, layout="time")
    rng = np.random.default_rng(3)
    arm_cf = rng.integers(0, 2, (N, T)).astype(np.int8)
    bits = ops.pack_arm_bits(torch.tensor(np.ascontiguousarray(arm_cf.T), device=dev), N)
    y0 = torch.tensor(g["x"][:, 0].copy(), device=dev)
    fc = torch.empty((N, 2, lib.n_terms), dtype=torch.float64, device=dev)
    fm = torch.empty((N, lib.n_terms), dtype=torch.int8, device=dev)
    fi = torch.empty((N,), dtype=torch.int32, device=dev)
    y = ops.refit_rollout_moments(mom, u, arm, rows, T, lib, coef, 0.1, 0.5, y0, bits, dt, T, fits=(fc, fm, fi))
    torch.cuda.synchronize()
    c_glob = coef.cpu().numpy()
    pc_ref, pm_ref, pi_ref = R.per_patient_fit(g["x"], g["u"], g["arm"], g["rows"], dt, exps, c_glob, 0.1, 0.5)
    np.testing.assert_array_equal(fm.cpu().numpy(), pm_ref)
    np.testing.assert_array_equal(fi.cpu().numpy(), pi_ref)
    assert np.abs(fc.cpu().numpy() - pc_ref).max() < 1e-8
    y_ref = R.rollout(g["x"][:, 0], g["u"], arm_cf.astype(np.int64), pc_ref, exps, dt, "euler5")
    np.testing.assert_allclose(y.cpu().numpy().T, y_ref, rtol=1e-10, atol=1e-10)


def test_fold_matches_oracle_sampled_at_config_size(dev):
    """The C4 bench's cohort (1M x 60, seed as bench.py c4_main rank 0): refits and trajectories of a
    1,500-patient sample (first and last tiles included) against the row-form oracle."""
    from insite_amd import cohort, ops
    N, T, seed = 1_000_000, 60, 1003
    coh = cohort.synthetic_pkpd(N, T, seed=seed, device=dev, equation="EQ_4_C", layout="time")
    lib = coh.lib
    exps = lib.exps.astype(np.int64)
    coef, _, _, _, _, mom = ops.gram_moments(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, layout="time")
    bits = cohort.counterfactual_arms(coh.arm, T, seed=seed, layout="time_bits")
    fc = torch.empty((N, 2, lib.n_terms), dtype=torch.float64, device=dev)
    fm = torch.empty((N, lib.n_terms), dtype=torch.int8, device=dev)
    fi = torch.empty((N,), dtype=torch.int32, device=dev)
    y = ops.refit_rollout_moments(mom, coh.u, coh.arm, coh.rows, T, lib, coef, 0.1, 0.5, coh.y0, bits, coh.dt, T,
                                  fits=(fc, fm, fi))
    torch.cuda.synchronize()
    rng = np.random.default_rng(seed)
    idx = np.unique(np.concatenate([np.arange(64), np.arange(N - 64, N), rng.choice(N, 1372, replace=False)]))
    it = torch.as_tensor(idx, device=dev)
    xs = coh.x[:T].index_select(1, it).t().contiguous().cpu().numpy()
    us = coh.u.index_select(0, it).cpu().numpy()
    ars = coh.arm.index_select(0, it).cpu().numpy().astype(np.int64)
    rws = coh.rows.index_select(0, it).cpu().numpy()
    pc_ref, pm_ref, pi_ref = R.per_patient_fit(xs, us, ars, rws, coh.dt, exps, coef.cpu().numpy(), 0.1, 0.5)
    np.testing.assert_array_equal(fm.index_select(0, it).cpu().numpy(), pm_ref)
    np.testing.assert_array_equal(fi.index_select(0, it).cpu().numpy(), pi_ref)
    assert np.abs(fc.index_select(0, it).cpu().numpy() - pc_ref).max() < 1e-8
    # the sampled patients' counterfactual arms, unpacked from the bit rows
    words = bits.cpu().numpy().astype(np.uint32)                       # [T, ceil(N / 32)]
    arm_cf = ((words[:, idx >> 5] >> (idx & 31).astype(np.uint32)) & 1).T.astype(np.int64)
    y_ref = R.rollout(coh.y0.index_select(0, it).cpu().numpy(), us, arm_cf, pc_ref, exps, coh.dt, "euler5")
    np.testing.assert_allclose(y.index_select(1, it).cpu().numpy().T, y_ref, rtol=1e-10, atol=1e-10)


def test_fold_refuses_unsupported(dev):
    from insite_amd import _lib, cohort, ops
    N, T = 256, 20
    coh = cohort.synthetic_pkpd(N, T, seed=5, device=dev, equation="EQ_4_C", layout="time")
    coef, _, _, _, _, mom = ops.gram_moments(coh.x, coh.u, coh.arm, coh.rows, coh.dt, coh.lib, 0.1, 0.5, layout="time")
    bits = cohort.counterfactual_arms(coh.arm, T, seed=5, layout="time_bits")
    with pytest.raises(_lib.InsiteError):            # alpha = 0: the closed form needs a ridge
        ops.refit_rollout_moments(mom, coh.u, coh.arm, coh.rows, T, coh.lib, coef, 0.1, 0.0, coh.y0, bits, coh.dt, T)
    with pytest.raises(ValueError):
        ops.refit_rollout_moments(mom.cpu(), coh.u, coh.arm, coh.rows, T, coh.lib, coef, 0.1, 0.5, coh.y0, bits,
                                  coh.dt, T)
