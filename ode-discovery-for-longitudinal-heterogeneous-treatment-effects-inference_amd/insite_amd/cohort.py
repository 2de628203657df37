"""On-device PK/PD cohort generation (input side of the hot path).

Distributions follow ``get_standard_params`` / ``simulate_factual``
(``libs_m/ct/src/data/pkpd/pkpd_simulation.py:96-203, 205-309``): c_a ~ N(0.5, 0.05),
x0 ~ U(1, 50), C_a = c_a (EQ_4_A/B) or c_0 + 0.05 / c_1 + 0.15 (EQ_4_C/D; EQ_4_D adds one
N(0, 0.25) shift per arm), treatment ~ Bernoulli(sigmoid(gamma/50 (x0 - 25))), volumes are the
Euler-5 trajectory of dy/dt = -C_a y, plus 0.01 N(0,1) noise for B/C/D.  The trajectories are
integrated by the same HIP rollout kernel the model uses (per-patient coefficient rows carrying
the true -C_a on the ``x0`` column), so no host round trip is needed for multi-GPU shards.
Random numbers come from torch's device generator (the reference's JAX threefry streams are not
reproducible without jax).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import ops
from .library import PolyLibrary, polynomial_library

MAX_VALUE = 50.0
MAX_TIME_HORIZON = 10.0
OBSERVATION_NOISE = 0.01


@dataclass
class DeviceCohort:
    x: torch.Tensor          # volume series: [N, ldx] (layout "patient") or [T, ldx >= N] ("time")
    u: torch.Tensor          # [N, 2] f64 statics (c_0, c_1)
    arm: torch.Tensor        # [N] int8 factual (training) arm
    rows: torch.Tensor       # [N] int32 discovery rows per patient (seq_len - 1)
    C: torch.Tensor          # [N, 2] f64 hidden rates
    T: int
    dt: float
    lib: PolyLibrary
    layout: str = "patient"

    @property
    def y0(self) -> torch.Tensor:
        return (self.x[0, : self.arm.numel()] if self.layout == "time" else self.x[:, 0]).contiguous()


def _gen(seed: int, device) -> torch.Generator:
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    return g


def synthetic_pkpd(n_patients: int, T: int, seed: int, device, equation: str = "EQ_4_C",
                   conf_coeff: float = 2.0, noise: bool | None = None, layout: str = "patient") -> DeviceCohort:
    """Cohort of ``n_patients`` factual trajectories of T observations.  layout "patient": x is
    [N, T + (T & 1)]; layout "time": x is [T, round_up(N, 2)] (one contiguous run per step)."""
    dev = torch.device(device)
    g = _gen(seed, dev)
    N = int(n_patients)
    f64 = torch.float64
    c = torch.randn((N, 2), generator=g, device=dev, dtype=f64) * 0.05 + 0.5
    C = c.clone()
    if equation in ("EQ_4_C", "EQ_4_D"):
        C[:, 0] += 0.05
        C[:, 1] += 0.15
        if equation == "EQ_4_D":
            C += torch.randn((1, 2), generator=g, device=dev, dtype=f64) * 0.25
    elif equation not in ("EQ_4_A", "EQ_4_B"):
        raise NotImplementedError(equation)
    x0 = torch.rand((N,), generator=g, device=dev, dtype=f64) * (MAX_VALUE - 1.0) + 1.0
    prob = torch.sigmoid((conf_coeff / MAX_VALUE) * (x0 - MAX_VALUE / 2.0))
    arm = (torch.rand((N,), generator=g, device=dev, dtype=f64) < prob).to(torch.int8)
    lib = polynomial_library(2, 2, True)
    dt = MAX_TIME_HORIZON / T
    coef = torch.zeros((N, 2, lib.n_terms), device=dev, dtype=f64)
    coef[:, :, 1] = -C                               # 'x0' column carries -C_a
    if layout == "time":
        ld = N + (N & 1)
        x = torch.zeros((T, ld), device=dev, dtype=f64)
        x[0, :N] = x0
        lda = (N + 3) // 4 * 4
        arms = torch.empty((max(T - 1, 1), lda), dtype=torch.int8, device=dev)
        arms[:, :N] = arm[None, :]
        arms[:, N:] = 0
        if T > 1:
            ops.rollout(x0, c.contiguous(), arms, coef, lib, dt, method="euler5", drop_below=0.0, T=T - 1,
                        out=x[1:T], layout="time")
        if noise if noise is not None else equation.split("_")[-1] in ("B", "C", "D"):
            x[:, :N] += OBSERVATION_NOISE * torch.randn((T, N), generator=g, device=dev, dtype=f64)
    elif layout == "patient":
        ldx = T + (T & 1)
        x = torch.empty((N, ldx), device=dev, dtype=f64)
        x[:, 0] = x0
        if ldx > T:
            x[:, T:] = 0.0
        lda = (T + 15) // 16 * 16
        arms = torch.empty((N, lda), dtype=torch.int8, device=dev)
        arms[:] = arm[:, None]
        if T > 1:
            ops.rollout(x0, c.contiguous(), arms, coef, lib, dt, method="euler5", drop_below=0.0, T=T - 1,
                        out=x[:, 1:T])
        if noise if noise is not None else equation.split("_")[-1] in ("B", "C", "D"):
            x[:, :T] += OBSERVATION_NOISE * torch.randn((N, T), generator=g, device=dev, dtype=f64)
    else:
        raise ValueError(f"layout {layout!r}")
    rows = torch.full((N,), T - 2, device=dev, dtype=torch.int32)   # seq_len = T-1, offset 1
    return DeviceCohort(x=x, u=c.contiguous(), arm=arm, rows=rows, C=C, T=T, dt=dt, lib=lib, layout=layout)


def counterfactual_arms(arm: torch.Tensor, T: int, seed: int, layout: str = "patient") -> torch.Tensor:
    """Per-step arm sequences: the factual arm, flipped from a random step on (C2 workload).

    layout "patient": [N, round_up(T, 16)] (16-byte rows: the patient-major rollout reads 16 B per
    lane); layout "time": [T, round_up(N, 4)] (time-major; 4-byte rows let the rollout load
    dwords); layout "time_bits": int32 [T, ceil(N/32)] bitmask (ops.pack_arm_bits); "tile_bits": the same bits
    tile-major, int32 [ceil(N/64), T, 2] (ops.tile_major_bits)."""
    dev = arm.device
    g = _gen(seed + 7919, dev)
    N = arm.numel()
    flip = torch.randint(0, T, (N, 1), generator=g, device=dev)
    steps = torch.arange(T, device=dev)[None, :]
    seq = torch.where(steps >= flip, 1 - arm[:, None], arm[:, None]).to(torch.int8)
    if layout in ("time", "time_bits", "tile_bits"):
        ld = (N + 3) // 4 * 4
        out = torch.zeros((T, ld), dtype=torch.int8, device=dev)
        out[:, :N] = seq.t()
        if layout == "time_bits":
            from .ops import pack_arm_bits
            return pack_arm_bits(out, N)
        if layout == "tile_bits":
            from .ops import pack_arm_bits, tile_major_bits
            return tile_major_bits(pack_arm_bits(out, N), N)
        return out
    lda = (T + 15) // 16 * 16
    out = torch.empty((N, lda), dtype=torch.int8, device=dev)
    out[:, :T] = seq
    if lda > T:
        out[:, T:] = 0
    return out


def irregular_grid(n_patients: int, seed: int, device, t_max: float = MAX_TIME_HORIZON, n_min: int = 20,
                   n_max: int = 60):
    """C5 observation grids on device (oracle/rk45_ref.irregular_grid distribution): T_p ~ U{n_min..n_max},
    t_0 = 0 and T_p - 1 sorted U(0, t_max) times.  Returns (t_obs [n_max, N] f64 time-major — rows past
    a patient's grid are NaN —, n_obs [N] int32)."""
    dev = torch.device(device)
    g = _gen(seed, dev)
    N = int(n_patients)
    n_obs = torch.randint(n_min, n_max + 1, (N,), generator=g, device=dev, dtype=torch.int32)
    r = torch.rand((n_max - 1, N), generator=g, device=dev, dtype=torch.float64) * t_max
    k = torch.arange(n_max - 1, device=dev)[:, None]
    r = torch.where(k < (n_obs[None, :] - 1), r, torch.full_like(r, float("inf")))
    r, _ = torch.sort(r, dim=0)
    t = torch.empty((n_max, N), dtype=torch.float64, device=dev)
    t[0] = 0.0
    t[1:] = torch.where(torch.isinf(r), torch.full_like(r, float("nan")), r)
    return t.contiguous(), n_obs


@dataclass
class SegmentCohort:
    x: torch.Tensor          # [T + 1, N] f64 time-major samples (x[0] = y0)
    u: torch.Tensor          # [N, U] f64 statics
    arm: torch.Tensor        # [T, round_up(N, 4)] int8 time-major per-step arm (4 arms)
    seq_len: torch.Tensor    # [N] int32
    T: int
    dt: float
    lib: PolyLibrary


def markov_arms(n_patients: int, T: int, n_arms: int, switch_p: float, g: torch.Generator, device) -> torch.Tensor:
    """Per-step treatment sequences [T, round_up(N, 4)] int8 (time-major): a uniformly drawn first arm,
    then with probability ``switch_p`` per step a switch to a uniformly drawn other arm."""
    N = int(n_patients)
    ld = (N + 3) // 4 * 4
    out = torch.zeros((T, ld), dtype=torch.int8, device=device)
    a = torch.randint(0, n_arms, (N,), generator=g, device=device)
    for k in range(T):
        if k:
            sw = torch.rand((N,), generator=g, device=device) < switch_p
            other = (a + torch.randint(1, max(n_arms, 2), (N,), generator=g, device=device)) % n_arms
            a = torch.where(sw, other, a)
        out[k, :N] = a.to(torch.int8)
    return out


def synthetic_segments(n_patients: int, T: int, seed: int, device, coef, n_statics: int = 1, switch_p: float = 0.1,
                       noise: float = OBSERVATION_NOISE, dt: float = 0.1) -> SegmentCohort:
    """A 4-arm cohort with the layout of the cancer_sim / EQ_5 datasets (the reference
    simulators themselves, data/cancer_sim and data/continuous/continuous.py, are not on the path): the
    planted per-arm model ``coef`` [A, F] over the degree-2 interaction library of [x0, statics] is
    integrated with the Euler-5 rollout kernel under Markov per-step arms, plus observation noise."""
    dev = torch.device(device)
    g = _gen(seed, dev)
    N = int(n_patients)
    f64 = torch.float64
    lib = polynomial_library(n_statics, 2, True)
    c = torch.as_tensor(coef, dtype=f64, device=dev).contiguous()
    u = (torch.randn((N, n_statics), generator=g, device=dev, dtype=f64) * 0.05 + 0.5).contiguous()
    y0 = torch.rand((N,), generator=g, device=dev, dtype=f64) * 4.0 + 1.0
    arms = markov_arms(N, T, c.size(0), switch_p, g, dev)
    x = torch.empty((T + 1, N), dtype=f64, device=dev)
    x[0] = y0
    ops.rollout(y0, u, arms, c, lib, dt, method="euler5", drop_below=0.0, T=T, out=x[1:], layout="time")
    if noise:
        x += noise * torch.randn((T + 1, N), generator=g, device=dev, dtype=f64)
    sl = torch.full((N,), T, dtype=torch.int32, device=dev)
    return SegmentCohort(x=x, u=u, arm=arms, seq_len=sl, T=T, dt=dt, lib=lib)
