"""C4's two fits from one pass over x (ABI 4): insite_gram_moments_f64 (Gram + global STLSQ + every
patient's moments) and insite_fit_per_patient_moments_f64 must give what insite_sindy_fit_f64 and
insite_sindy_fit_per_patient_f64 give (those are pinned to the oracle in test_gpu_parity.py):
G/b to rtol 1e-12 (fixed-order sums over a different item split), identical global and per-patient
supports, coefficient L-inf < 1e-10, per-patient iteration counts equal -- both layouts, ragged rows
(incl. < 5: no contribution, global model kept), and the N > 1 form (Gram + moments, then STLSQ)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,T,layout,ragged", [(100_000, 60, "time", False), (3_001, 60, "time", True),
                                               (2_000, 37, "patient", True), (125_000, 500, "time", False)])
def test_one_pass_fits_match_two_pass(dev, N, T, layout, ragged):
    from insite_amd import cohort, ops
    coh = cohort.synthetic_pkpd(N, T, seed=7, device=dev, equation="EQ_4_C", layout=layout)
    rows = coh.rows
    if ragged:
        g = torch.Generator(device=dev)
        g.manual_seed(N)
        rows = torch.randint(0, T - 1, (N,), generator=g, device=dev, dtype=torch.int32)
    lib = coh.lib
    coef, mask, iters, G, b, mom = ops.gram_moments(coh.x, coh.u, coh.arm, rows, coh.dt, lib, 0.1, 0.5,
                                                    layout=layout)
    pc, pm, pi = ops.fit_per_patient_moments(mom, coh.u, coh.arm, rows, T, lib, coef, 0.1, 0.5)
    c2, m2, i2, G2, b2 = ops.sindy_fit(coh.x, coh.u, coh.arm, rows, coh.dt, lib, 0.1, 0.5, layout=layout)
    pc2, pm2, pi2 = ops.sindy_fit_per_patient(coh.x, coh.u, coh.arm, rows, coh.dt, lib, c2, 0.1, 0.5, layout=layout)
    torch.cuda.synchronize()
    np.testing.assert_allclose(G.cpu().numpy(), G2.cpu().numpy(), rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(b.cpu().numpy(), b2.cpu().numpy(), rtol=1e-12, atol=1e-9)
    assert torch.equal(mask, m2) and (coef - c2).abs().max().item() < 1e-10
    assert torch.equal(pm, pm2) and torch.equal(pi, pi2)
    assert (pc - pc2).abs().max().item() < 1e-10
    # moments: rows count and sums per patient (rows < 5 contribute nothing)
    L = torch.clamp(rows, max=T).to(torch.float64)
    L = torch.where(L < 5, torch.zeros_like(L), L)
    assert torch.equal(mom[:, 0], L)
    # N > 1 form: Gram + moments without the fused STLSQ, then the replicated STLSQ on (G, b)
    _, _, _, G3, b3, mom3 = ops.gram_moments(coh.x, coh.u, coh.arm, rows, coh.dt, lib, None, layout=layout)
    c3, m3, _ = ops.stlsq(G3, b3, 0.1, 0.5)
    torch.cuda.synchronize()
    np.testing.assert_allclose(G3.cpu().numpy(), G.cpu().numpy(), rtol=1e-13, atol=1e-10)
    np.testing.assert_allclose(mom3.cpu().numpy(), mom.cpu().numpy(), rtol=1e-13, atol=1e-10)
    assert torch.equal(m3, mask)
    assert (c3 - coef).abs().max().item() < 1e-10
