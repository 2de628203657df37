"""Multi-state path (BASELINE.json configuration C3): S coupled states + one binary per-step treatment.

Torch front end of ``insite_gram_ms_f32`` / ``insite_stlsq_wave_f64`` / ``insite_rollout_ms_f32``
(include/insite_hip.h).  C3 is build-defined — the reference has no multi-state system — and extends the
reference's discovery semantics (SINDy + SmoothedFiniteDifference + PolynomialLibrary + STLSQ,
libs_m/ct/src/models/sindy.py:186-213) and its rollout (odeint, pkpd/utils.py:68-94) to S states; the
restatement it is checked against is oracle/multistate_ref.py.

Layouts (time-major structure of arrays):
    x      [T, S, >=N] float32      step k, state s, patient p
    a      [T, >=ceil(N/32)] int32  TIME_MAJOR_BITS treatment mask (ops.pack_arm_bits)
    y0     [S, >=N] float32
    y      [T, S, >=N] float32      state after interval k
No CPU fallback: device tensors only; a missing library raises InsiteLibraryError.
"""
from __future__ import annotations

import ctypes
import itertools
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from .ops import METHODS, Workspace, _default_ws, _ws, _dev, _p, _stream, pack_arm_bits

RATES_C3 = {"k1": 1.2, "k2": 0.8, "k3": 0.5, "k4": 0.6, "k5": 0.1, "e": 0.4, "D": 2.0}
THRESHOLD_C3 = 0.05
ALPHA_C3 = 0.5
DT_C3 = 0.02


@dataclass(frozen=True)
class MsLibrary:
    """pysindy PolynomialLibrary(degree 2) over (x_1..x_S, a_1..a_NIN), states first."""
    exps: np.ndarray       # int8 [F, S + NIN]
    n_states: int
    n_inputs: int

    @property
    def n_terms(self) -> int:
        return int(self.exps.shape[0])

    def names(self):
        inputs = [f"x{i + 1}" for i in range(self.n_states)] + (["a"] if self.n_inputs else [])
        out = []
        for e in self.exps:
            parts = [n if k == 1 else f"{n}^{int(k)}" for n, k in zip(inputs, e) if k]
            out.append(" ".join(parts) if parts else "1")
        return out

    def table(self) -> np.ndarray:
        return np.ascontiguousarray(self.exps, dtype=np.int8)


def ms_library(n_states: int = 5, n_inputs: int = 1, interaction_only: bool = True) -> MsLibrary:
    n = n_states + n_inputs
    comb = itertools.combinations if interaction_only else itertools.combinations_with_replacement
    rows = []
    for deg in range(0, 3):
        for c in comb(range(n), deg):
            e = [0] * n
            for i in c:
                e[i] += 1
            rows.append(e)
    return MsLibrary(np.array(rows, dtype=np.int8), n_states, n_inputs)


def c3_truth_coef(lib: MsLibrary, rates=RATES_C3, device=None) -> torch.Tensor:
    """True C3 coefficients [S, F] in the library basis (oracle/multistate_ref.c3_truth_coef):
    x1' = -k1 x1 + D a, x2' = k1 x1 - k2 x2, x3' = k2 x2 - k3 x3, x4' = k3 x3 - k4 x4,
    x5' = -k5 x5 - e x4 x5."""
    E = lib.exps.astype(np.int64)

    def col(*idx):
        e = np.zeros(E.shape[1], dtype=np.int64)
        for i in idx:
            e[i] += 1
        return int(np.nonzero((E == e).all(axis=1))[0][0])

    k = rates
    C = np.zeros((5, E.shape[0]))
    C[0, col(0)], C[0, col(5)] = -k["k1"], k["D"]
    C[1, col(0)], C[1, col(1)] = k["k1"], -k["k2"]
    C[2, col(1)], C[2, col(2)] = k["k2"], -k["k3"]
    C[3, col(2)], C[3, col(3)] = k["k3"], -k["k4"]
    C[4, col(4)], C[4, col(3, 4)] = -k["k5"], -k["e"]
    return torch.tensor(C, dtype=torch.float64, device=device)


def _check_x(x: torch.Tensor, S: int):
    _dev("x", x, torch.float32, 3)
    if x.size(1) != S or x.stride(1) != x.size(2) or x.stride(0) != S * x.size(2):
        raise ValueError("x must be a contiguous [T, S, ldx] float32 tensor")


def _check_bits(a, N, T):
    if a is None:
        return ctypes.c_void_p(0), 0
    _dev("a", a, torch.int32, 2)
    if a.size(1) < (N + 31) // 32 or a.size(0) < T:
        raise ValueError("treatment bits must be [>=T, >=ceil(N/32)] int32")
    return _p(a), a.stride(0)


def gram_ms(x: torch.Tensor, a: torch.Tensor | None, lib: MsLibrary, dt: float, rows: torch.Tensor | None = None,
            n_patients: int | None = None, workspace: Workspace | None = None, out: tuple | None = None):
    """G [F, F], B [F, S] of the multi-state regression (insite_gram_ms_f32).  x [T, S, ldx] float32,
    a TIME_MAJOR_BITS int32 [T, W] or None (library over the states only), rows [N] int32 or None."""
    L = _lib.load()
    S = lib.n_states
    _check_x(x, S)
    T, ldx = x.size(0), x.size(2)
    N = ldx if n_patients is None else int(n_patients)
    if (a is None) != (lib.n_inputs == 0):
        raise ValueError("the library's input column needs the treatment bits (and vice versa)")
    ap, lda = _check_bits(a, N, T)
    if rows is not None:
        _dev("rows", rows, torch.int32, 1)
        if rows.numel() != N:
            raise ValueError("rows must have one entry per patient")
    dev = x.device
    F = lib.n_terms
    if out is None:
        out = (torch.empty((F, F), dtype=torch.float64, device=dev), torch.empty((F, S), dtype=torch.float64, device=dev))
    G, B = out
    ws = _ws(workspace, dev, "scratch").get(L.insite_gram_ms_workspace_bytes(N), dev)
    tab = lib.table()
    st = L.insite_gram_ms_f32(_p(x), ldx, T, S, ap, lda, _p(rows), N, tab.ctypes.data_as(ctypes.c_void_p), F, 0,
                              float(dt), _p(G), _p(B), _p(ws), ws.numel(), _stream(dev))
    _lib.check("insite_gram_ms_f32", st)
    return G, B


def stlsq_wave(G: torch.Tensor, B: torch.Tensor, threshold: float, alpha: float, max_iter: int = 100,
               unbias: bool = True, out: tuple | None = None):
    """One STLSQ per target column of B on the shared Gram G (insite_stlsq_wave_f64, F <= 32).
    Returns (coef [S, F], mask [S, F], iters [S])."""
    L = _lib.load()
    _dev("G", G, torch.float64, 2)
    _dev("B", B, torch.float64, 2)
    F, S = B.shape
    if G.shape != (F, F) or not G.is_contiguous() or not B.is_contiguous():
        raise ValueError("G [F, F] and B [F, S] must be contiguous")
    if out is None:
        out = (torch.empty((S, F), dtype=torch.float64, device=G.device),
               torch.empty((S, F), dtype=torch.int8, device=G.device),
               torch.empty((S,), dtype=torch.int32, device=G.device))
    coef, mask, iters = out
    st = L.insite_stlsq_wave_f64(_p(G), _p(B), F, S, float(threshold), float(alpha), int(max_iter),
                                 int(bool(unbias)), _p(coef), _p(mask), _p(iters), _stream(G.device))
    _lib.check("insite_stlsq_wave_f64", st)
    return out


def fit_ms(x, a, lib: MsLibrary, dt: float, threshold: float = THRESHOLD_C3, alpha: float = ALPHA_C3,
           rows=None, n_patients=None, workspace=None):
    """Discovery of the S-state model: Gram pass + one STLSQ per state.  Returns (coef, mask, iters, G, B)."""
    G, B = gram_ms(x, a, lib, dt, rows, n_patients, workspace)
    coef, mask, iters = stlsq_wave(G, B, threshold, alpha)
    return coef, mask, iters, G, B


def rollout_ms(y0: torch.Tensor, a: torch.Tensor | None, coef: torch.Tensor, lib: MsLibrary, dt: float,
               T: int, method: str = "rk4", substeps: int | None = None, drop_below: float = 1e-3,
               out: torch.Tensor | None = None, n_rows: int | None = None, support=None):
    """S-state open-loop rollout (insite_rollout_ms_f32).  y0 [S, >=N] float32, a bits [T, W] or None,
    coef [S, F] f64.  Returns y [T, S, N] float32 (state after each interval).

    ``support`` (host [S, F] bool/int, e.g. the STLSQ mask): the support-specialised kernel
    (insite_rollout_ms_sparse_f32, generated with hipRTC on first use per support) — same results, only
    the model's terms evaluated; a coefficient outside ``support`` makes that launch run the dense RHS."""
    L = _lib.load()
    S = lib.n_states
    _dev("y0", y0, torch.float32, 2)
    if y0.size(0) != S:
        raise ValueError("y0 must be [S, N]")
    N = y0.size(1) if n_rows is None else int(n_rows)
    ap, lda = _check_bits(a, N, T)
    _dev("coef", coef, torch.float64, 2)
    if tuple(coef.shape) != (S, lib.n_terms) or not coef.is_contiguous():
        raise ValueError("coef must be a contiguous [S, F] f64 tensor")
    m, default_sub = METHODS[method]
    sub = int(substeps or default_sub)
    if out is None:
        out = torch.empty((T, S, N), dtype=torch.float32, device=y0.device)
    else:
        _check_x(out, S)
        if out.size(0) < T or out.size(2) < N:
            raise ValueError("out must be [>=T, S, >=N]")
    tab = lib.table()
    if support is not None:
        sup = np.ascontiguousarray(np.asarray(support) != 0, dtype=np.int8)
        if sup.shape != (S, lib.n_terms):
            raise ValueError("support must be a host [S, F] mask")
        st = L.insite_rollout_ms_sparse_f32(_p(y0), y0.stride(0), ap, lda, _p(coef), sup.ctypes.data_as(ctypes.c_void_p),
                                            tab.ctypes.data_as(ctypes.c_void_p), lib.n_terms, S, N, int(T), float(dt), m,
                                            sub, float(drop_below), _p(out), out.size(2), _stream(y0.device))
        _lib.check("insite_rollout_ms_sparse_f32", st)
        return out
    st = L.insite_rollout_ms_f32(_p(y0), y0.stride(0), ap, lda, _p(coef), tab.ctypes.data_as(ctypes.c_void_p),
                                 lib.n_terms, S, N, int(T), float(dt), m, sub, float(drop_below), _p(out),
                                 out.size(2), _stream(y0.device))
    _lib.check("insite_rollout_ms_f32", st)
    return out


def markov_treatment_bits(N: int, T: int, generator: torch.Generator, device, p1: float = 0.3,
                          p_switch: float = 0.01) -> torch.Tensor:
    """Per-step binary treatment: a_0 ~ Bernoulli(p1), switching with probability p_switch per step
    (oracle/multistate_ref.treatment_markov distribution); returned packed, [T, ceil(N/32)] int32."""
    a0 = (torch.rand((N,), generator=generator, device=device) < p1).to(torch.int32)
    sw = (torch.rand((T, N), generator=generator, device=device) < p_switch).to(torch.int32)
    sw[0] = 0
    flips = torch.cumsum(sw, dim=0, dtype=torch.int32)
    arm = ((a0[None, :] + flips) & 1).to(torch.int8)
    del sw, flips
    return pack_arm_bits(arm, N)


@dataclass
class C3Cohort:
    x: torch.Tensor       # [T, S, N] float32 observations (x[0] = initial state)
    a: torch.Tensor       # [T, W] int32 treatment bits
    lib: MsLibrary
    dt: float

    @property
    def y0(self) -> torch.Tensor:
        return self.x[0]


def synthetic_c3(N: int, T: int, seed: int, device, dt: float = DT_C3, substeps: int = 10) -> C3Cohort:
    """On-device C3 cohort: x1..x4 ~ U(0, 1), x5 ~ U(1, 5), Markov treatments, trajectories integrated by
    the rollout kernel with the TRUE coefficients and ``substeps`` RK4 steps per interval (the data
    generator shares the model's integrator, as the PK/PD generator does)."""
    dev = torch.device(device)
    g = torch.Generator(device=dev)
    g.manual_seed(int(seed))
    lib = ms_library(5, 1, True)
    x = torch.empty((T, 5, N), dtype=torch.float32, device=dev)
    lo = torch.tensor([0, 0, 0, 0, 1], dtype=torch.float32, device=dev)[:, None]
    span = torch.tensor([1, 1, 1, 1, 4], dtype=torch.float32, device=dev)[:, None]
    x[0] = lo + span * torch.rand((5, N), generator=g, device=dev)
    a = markov_treatment_bits(N, T, g, dev)
    if T > 1:
        rollout_ms(x[0], a, c3_truth_coef(lib, device=dev), lib, dt, T - 1, method="rk4", substeps=substeps,
                   drop_below=0.0, out=x[1:], n_rows=N)
    return C3Cohort(x, a, lib, dt)
