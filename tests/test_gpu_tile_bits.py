"""Tile-major bit arms (round 6; insite_hip.h ``INSITE_ARM_BITS_TILE_MAJOR``, ``ops.tile_major_bits``): the same
per-step arm bits as TIME_MAJOR_BITS, stored [ceil(N/64), S >= T, 2] int32 so that a 64-patient tile's 32-step
group is one 256-byte run (the time-major rows put 16 tiles on one 128-B line, which a 1M-patient rollout re-fetched
once per tile: PMC 1.12x of the north-star step's algorithmic bytes).  A layout only: every rollout that reads bits
through rollout_bits_range -- insite_rollout_f64, the fused / deferred / lagged steps, the C4 refit rollout -- must
give results bitwise equal to the time-major form's, including partial last tiles (N % 64 in (0, 32] and (32, 64)),
T not a multiple of the 32-step group, and a padded S > T."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _arms(dev, N, T, seed):
    from insite_amd import cohort
    coh = cohort.synthetic_pkpd(N, T, seed=seed, device=dev, equation="EQ_4_C", layout="time")
    bits = cohort.counterfactual_arms(coh.arm, T, seed=seed, layout="time_bits")
    tiles = cohort.counterfactual_arms(coh.arm, T, seed=seed, layout="tile_bits")
    return coh, bits, tiles


@pytest.mark.parametrize("N,T", [(1, 5), (20, 33), (100, 64), (4_127, 77), (65_535, 200)])
def test_tile_major_bits_hold_the_same_arms(dev, N, T):
    """tile word (t, k, h) bit j == time-major word (k, 2t + h) bit j for every stored patient."""
    from insite_amd import ops
    _, bits, tiles = _arms(dev, N, T, 5)
    assert tiles.shape == ((N + 63) // 64, T, 2) and tiles.dtype == torch.int32 and tiles.is_contiguous()
    W = (N + 31) // 32
    tm = tiles.permute(1, 0, 2).reshape(T, -1)[:, :W]
    assert torch.equal(tm, bits[:, :W])
    # padded steps per tile (S > T) through the public helper
    padded = torch.zeros((T + 7, bits.size(1)), dtype=torch.int32, device=dev)
    padded[:T] = bits
    t2 = ops.tile_major_bits(padded, N)
    assert torch.equal(t2[:, :T], tiles)


@pytest.mark.parametrize("N,T", [(20, 33), (100, 64), (4_127, 77), (65_535, 200)])
def test_rollout_tile_bits_equals_time_bits(dev, N, T):
    from insite_amd import ops
    coh, bits, tiles = _arms(dev, N, T, 7)
    lib = coh.lib
    coef = torch.zeros((2, lib.n_terms), dtype=torch.float64, device=dev)
    coef[0, 4], coef[1, 1], coef[1, 5] = -1.11, -0.146, -1.02
    for method in ("rk4", "euler5"):
        y1 = ops.rollout(coh.y0, coh.u, bits, coef, lib, coh.dt, method=method, T=T, layout="time_bits")
        y2 = ops.rollout(coh.y0, coh.u, tiles, coef, lib, coh.dt, method=method, T=T, layout="time_bits")
        torch.cuda.synchronize()
        assert torch.equal(y1, y2)
    with pytest.raises(ValueError):   # S < T
        ops.rollout(coh.y0, coh.u, tiles[:, :T - 1].contiguous(), coef, lib, coh.dt, T=T, layout="time_bits")


@pytest.mark.parametrize("N,T", [(4_127, 77), (100_000, 200)])
def test_deferred_and_lagged_steps_tile_bits_equal_time_bits(dev, N, T):
    """The headline kernel's rollout role on tile-major bits: y bitwise the time-major run's, and the discovery
    roles untouched (G|b, models bitwise)."""
    from insite_amd import ops
    coh, bits, tiles = _arms(dev, N, T, 9)
    lib = coh.lib
    F = lib.n_terms
    cin = torch.zeros((2, F), dtype=torch.float64, device=dev)
    cin[0, 4], cin[1, 1], cin[1, 5] = -1.11, -0.146, -1.02
    res = []
    for arms in (bits, tiles):
        ws = ops.Workspace()
        o = tuple(torch.zeros(s, dtype=d, device=dev) for s, d in (((2, F), torch.float64), ((2, F), torch.int8),
                                                                    ((2,), torch.int32), ((2, F, F), torch.float64),
                                                                    ((2, F), torch.float64)))
        y = torch.empty((T, N), dtype=torch.float64, device=dev)
        for k in range(2):
            ops.fit_rollout_deferred(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, coh.y0, coh.u, arms, cin,
                                     coh.dt, k, k > 0, ws, T=T, y_out=y, out=o)
        yl = torch.empty((T, N), dtype=torch.float64, device=dev)
        wsl = ops.Workspace()
        Gr = torch.zeros((2, F, F), dtype=torch.float64, device=dev)
        br = torch.zeros((2, F), dtype=torch.float64, device=dev)
        for k in range(2):
            ops.plan_fit_rollout_lagged(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, coh.y0, coh.u, arms,
                                        cin, coh.dt, k, k > 0, wsl, (Gr, br), T=T, y_out=yl)()
        torch.cuda.synchronize()
        res.append((y.clone(), yl.clone()) + tuple(t.clone() for t in o) + (Gr.clone(), br.clone()))
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)
    assert np.all(np.isfinite(res[1][0].cpu().numpy()))


def test_refit_rollout_tile_bits_equal_time_bits(dev):
    from insite_amd import ops
    N, T = 3_001, 60
    coh, bits, tiles = _arms(dev, N, T, 11)
    lib = coh.lib
    coef, _, _, _, _, mom = ops.gram_moments(coh.x, coh.u, coh.arm, coh.rows, coh.dt, lib, 0.1, 0.5, layout="time")
    y1 = ops.refit_rollout_moments(mom, coh.u, coh.arm, coh.rows, T, lib, coef, 0.1, 0.5, coh.y0, bits, coh.dt, T)
    y2 = ops.refit_rollout_moments(mom, coh.u, coh.arm, coh.rows, T, lib, coef, 0.1, 0.5, coh.y0, tiles, coh.dt, T)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
