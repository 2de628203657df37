"""Torch-tensor front end of the C ABI (``include/insite_hip.h``).

Every op takes device tensors (contiguous rows; leading dimension = ``stride(0)``), launches on
torch's current HIP stream and returns without synchronising.  There is no CPU fallback: CPU
tensors raise ``ValueError`` and a missing library raises ``InsiteLibraryError``.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib
from .library import PolyLibrary

METHODS = {"euler5": (_lib.METHOD_EULER, 5), "euler": (_lib.METHOD_EULER, 1), "rk4": (_lib.METHOD_RK4, 1)}
FD_KINDS = {"smoothed4": _lib.FD_SMOOTHED4, "order4": _lib.FD_ORDER4}
LAYOUTS = {"patient": _lib.LAYOUT_PATIENT_MAJOR, "time": _lib.LAYOUT_TIME_MAJOR}
ROLLOUT_LAYOUTS = dict(LAYOUTS, time_bits=_lib.LAYOUT_TIME_MAJOR_BITS)


def pack_arm_bits(arm: torch.Tensor, n: int | None = None) -> torch.Tensor:
    """Time-major int8 arms [T, >=N] (values 0/1) -> the INSITE_LAYOUT_TIME_MAJOR_BITS bitmask
    int32 [T, ceil(N/32)]: bit (r & 31) of word r >> 5 is the arm of patient r.  Device-agnostic
    torch ops (data preparation, not on the hot path)."""
    T = arm.size(0)
    N = arm.size(1) if n is None else int(n)
    W = (N + 31) // 32
    a = torch.zeros((T, W * 32), dtype=torch.int64, device=arm.device)
    a[:, :N] = arm[:, :N].to(torch.int64)
    if bool((a > 1).any()):
        raise ValueError("bit-packed arms need n_arms <= 2 (arm values 0/1)")
    w = (a.view(T, W, 32) << torch.arange(32, device=arm.device, dtype=torch.int64)).sum(-1)
    w = torch.where(w >= 2 ** 31, w - 2 ** 32, w)
    return w.to(torch.int32).contiguous()


def tile_major_bits(bits: torch.Tensor, n: int) -> torch.Tensor:
    """Time-major bit arms int32 [T, >= ceil(n/32)] (``pack_arm_bits``) -> the tile-major form int32
    [ceil(n/64), T, 2] (insite_hip.h, ld_arm = INSITE_ARM_BITS_TILE_MAJOR(T)): a 64-patient tile's 32-step arm group
    is 256 contiguous bytes, where the time-major rows put 16 tiles on one 128-B line (re-fetched once per tile by a
    1M-patient rollout).  Data preparation, not on the hot path."""
    _dev("bits", bits, torch.int32, 2)
    T, W = bits.shape
    nt = (int(n) + 63) // 64
    if W < (int(n) + 31) // 32:
        raise ValueError("bits must be [T, >= ceil(n/32)] int32 words")
    w = torch.zeros((T, 2 * nt), dtype=torch.int32, device=bits.device)
    w[:, :min(W, 2 * nt)] = bits[:, :min(W, 2 * nt)]
    return w.view(T, nt, 2).permute(1, 0, 2).contiguous()


def _arm_bits_ld(arm_bits: torch.Tensor, N: int, T: int) -> int:
    """ld_arm of a bit-arm tensor: time-major [>= T, >= ceil(N/32)] int32 -> its row stride; tile-major
    [ceil(N/64), S >= T, 2] int32 (``tile_major_bits``) -> -S (insite_hip.h: INSITE_ARM_BITS_TILE_MAJOR)."""
    if arm_bits.dim() == 3:
        _dev("arm_bits", arm_bits, torch.int32, 3)
        if (arm_bits.size(0) != (N + 63) // 64 or arm_bits.size(1) < T or arm_bits.size(2) != 2
                or not arm_bits.is_contiguous()):
            raise ValueError("tile-major bit arms must be a contiguous [ceil(N/64), >= T, 2] int32 tensor")
        return -arm_bits.size(1)
    _dev("arm_bits", arm_bits, torch.int32, 2)
    if arm_bits.size(0) < T or arm_bits.size(1) < (N + 31) // 32:
        raise ValueError("arm_bits must be [T, >= ceil(N / 32)] int32 words (or tile-major [ceil(N/64), >= T, 2])")
    return arm_bits.stride(0)


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _dev(name, t, dtype, ndim=None):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ValueError(f"{name}: expected a device tensor (the INSITE HIP path has no CPU fallback)")
    if t.dtype != dtype:
        raise ValueError(f"{name}: expected {dtype}, got {t.dtype}")
    if ndim is not None and t.dim() != ndim:
        raise ValueError(f"{name}: expected {ndim}-d tensor, got shape {tuple(t.shape)}")
    if t.dim() >= 1 and t.size(-1) > 1 and t.stride(-1) != 1:   # a size-1 dimension may carry any stride
        raise ValueError(f"{name}: innermost dimension must be contiguous")
    if t.dim() == 2 and t.size(0) > 1 and t.stride(0) < t.size(1):
        raise ValueError(f"{name}: overlapping rows")
    return t


class Workspace:
    """Grow-only device scratch buffer (the library never allocates).  A buffer handed to a ``Plan`` is
    referenced by that plan, so growing the workspace later never frees memory a plan still writes to.
    Buffers start zeroed: the discovery kernels' arrival counters (the header) must be zero before a
    workspace's first use, and every call leaves them zero (insite_hip.h).  The invariant is enforced: a
    workspace takes the kind of the first op family it serves ("disc": gram / sindy_fit / segments /
    per-patient / fused step, whose header holds the counters; "scratch": ops that write from offset 0) and
    a later op of the other family raises ``ValueError`` instead of silently corrupting the counters."""

    def __init__(self, kind: str | None = None):
        self._buf = {}
        self.kind = kind

    def claim(self, kind: str) -> "Workspace":
        if self.kind is None:
            self.kind = kind
        elif self.kind != kind:
            raise ValueError(f"workspace serves the {self.kind!r} op family; a {kind!r} op would overwrite "
                             "its scratch (use a separate Workspace)")
        return self

    def get(self, nbytes: int, device) -> torch.Tensor:
        key = torch.device(device).index
        b = self._buf.get(key)
        if b is None or b.numel() < nbytes:
            b = torch.zeros(max(int(nbytes), 512), dtype=torch.uint8, device=device)
            self._buf[key] = b
        return b


# eager ops without an explicit workspace: one per (device, stream, kind), so launches on different
# streams never share scratch, and the discovery family ("disc": gram / sindy_fit / segments /
# per-patient, whose header holds the in-launch reduction's counters, zero between calls) never shares a
# buffer with ops that write scratch from offset 0
_WS_BY_STREAM: dict = {}


def _default_ws(device, kind: str = "scratch") -> Workspace:
    dev = torch.device(device)
    key = (dev.index, torch.cuda.current_stream(dev).cuda_stream, kind)
    ws = _WS_BY_STREAM.get(key)
    if ws is None:
        ws = _WS_BY_STREAM[key] = Workspace(kind)
    return ws


def _ws(workspace: Workspace | None, device, kind: str) -> Workspace:
    """The caller's workspace (claimed for ``kind``) or the per-stream default of that kind."""
    return workspace.claim(kind) if workspace is not None else _default_ws(device, kind)


def _plan_ws(workspace: Workspace | None) -> Workspace:
    """A plan of the discovery family: the caller's workspace (claimed) or a private one."""
    return workspace.claim("disc") if workspace is not None else Workspace("disc")


class Plan:
    """A prepared launch: arguments validated and packed once; the plan holds references to every
    tensor and host table its packed pointers address (inputs, outputs, workspace), so none can be freed
    while the plan lives.  Each call enqueues the kernel(s) on the current stream of the plan's device (or
    the given stream) with nothing but the C call left on the host path.  ``out`` holds the outputs.
    Plans made without a workspace get a private one (never the shared per-stream default)."""

    def __init__(self, fn_name: str, args: tuple, device, out, keep=()):
        self.fn_name = fn_name
        self._fn = getattr(_lib.load(), fn_name)
        self._args = args
        self._keep = tuple(keep)
        self.device = torch.device(device)
        self.out = out

    def __call__(self, stream: torch.cuda.Stream | None = None):
        h = (stream if stream is not None else torch.cuda.current_stream(self.device)).cuda_stream
        st = self._fn(*self._args, ctypes.c_void_p(h))
        if st:
            _lib.check(self.fn_name, st)
        return self.out

    def bind(self, stream: torch.cuda.Stream):
        """A zero-argument launcher with the stream handle packed too (hot loops: one C call).  The
        launcher keeps the plan (and so its tensors) alive."""
        fn, args, name = self._fn, self._args + (ctypes.c_void_p(stream.cuda_stream),), self.fn_name
        plan = self

        def launch():
            st = fn(*args)
            if st:
                _lib.check(name, st)
        launch.plan = plan
        return launch


def _run(prep):
    name, args, dev, out = prep[:4]
    st = getattr(_lib.load(), name)(*args, _stream(dev))
    _lib.check(name, st)
    return out


def _discovery_inputs(x, u, arm, rows, lib, layout):
    """Validate the discovery inputs; returns (N, n_steps, layout code)."""
    if layout not in LAYOUTS:
        raise ValueError(f"layout must be one of {sorted(LAYOUTS)}")
    _dev("x", x, torch.float64, 2)
    _dev("arm", arm, torch.int8, 1)
    _dev("rows", rows, torch.int32, 1)
    if layout == "time":
        N, n_steps = arm.numel(), x.size(0)
        if x.size(1) < N:
            raise ValueError("time-major x must be [n_steps, >= N]")
    else:
        N, n_steps = x.size(0), x.size(1)
    if lib.n_statics:
        _dev("u", u, torch.float64, 2)
        if u.size(0) != N or u.size(1) != lib.n_statics or u.stride(0) != lib.n_statics:
            raise ValueError("u must be a contiguous [N, n_statics] tensor")
    if arm.numel() != N or rows.numel() != N:
        raise ValueError("arm/rows must have one entry per patient")
    return N, n_steps, LAYOUTS[layout]


def _prep_gram(x, u, arm, rows, dt, lib, n_arms, fd, workspace, out, layout, stlsq_args=None):
    L = _lib.load()
    N, n_steps, lay = _discovery_inputs(x, u, arm, rows, lib, layout)
    F = lib.n_terms
    dev = x.device
    nbytes = L.insite_gram_workspace_bytes(N, n_arms, F)
    # workspace=False: validate and pack only (a caller that attaches its own workspace, e.g. the deferred step)
    ws = None if workspace is False else _ws(workspace, dev, "disc").get(nbytes, dev)
    wsp, wsn = (_p(ws), ws.numel()) if ws is not None else (ctypes.c_void_p(0), 0)
    tab = lib.ctypes_table()
    head = (_p(x), x.stride(0), lay, n_steps, _p(u) if lib.n_statics else ctypes.c_void_p(0), _p(arm), _p(rows), N,
            lib.n_statics, n_arms, tab.ctypes.data_as(ctypes.c_void_p), F, FD_KINDS[fd], float(dt))
    if stlsq_args is None:
        if out is None:
            out = (torch.empty((n_arms, F, F), dtype=torch.float64, device=dev),
                   torch.empty((n_arms, F), dtype=torch.float64, device=dev))
        G, b = out
        return "insite_gram_f64", head + (_p(G), _p(b), wsp, wsn), dev, out, (x, u, arm, rows, tab, ws, *out)
    threshold, alpha, max_iter, unbias = stlsq_args
    if out is None:
        out = (torch.empty((n_arms, F), dtype=torch.float64, device=dev),
               torch.empty((n_arms, F), dtype=torch.int8, device=dev),
               torch.empty((n_arms,), dtype=torch.int32, device=dev),
               torch.empty((n_arms, F, F), dtype=torch.float64, device=dev),
               torch.empty((n_arms, F), dtype=torch.float64, device=dev))
    coef, mask, iters, G, b = out
    args = head + (float(threshold), float(alpha), int(max_iter), int(bool(unbias)), _p(G), _p(b), _p(coef),
                   _p(mask), _p(iters), wsp, wsn)
    return "insite_sindy_fit_f64", args, dev, out, (x, u, arm, rows, tab, ws, *out)


def gram(x: torch.Tensor, u: torch.Tensor, arm: torch.Tensor, rows: torch.Tensor, dt: float,
         lib: PolyLibrary, n_arms: int = 2, fd: str = "smoothed4", workspace: Workspace | None = None,
         out: tuple | None = None, layout: str = "patient"):
    """Per-arm Gram G[A,F,F] and moments b[A,F] of the discovery regression (insite_gram_f64).

    layout "patient": x [N, T] (the reference's array); "time": x [T, >=N] (coalesced)."""
    return _run(_prep_gram(x, u, arm, rows, dt, lib, n_arms, fd, workspace, out, layout))


def sindy_fit(x: torch.Tensor, u: torch.Tensor, arm: torch.Tensor, rows: torch.Tensor, dt: float,
              lib: PolyLibrary, threshold: float, alpha: float, max_iter: int = 100, unbias: bool = True,
              n_arms: int = 2, fd: str = "smoothed4", workspace: Workspace | None = None,
              out: tuple | None = None, layout: str = "patient"):
    """Discovery in two launches (insite_sindy_fit_f64): Gram kernel, then the fixed-order
    reduction fused with one STLSQ fit per arm.  Replaces ``SINDy(...).fit`` per arm
    (reference sindy.py:190-192).  Returns (coef[A,F], mask[A,F], iters[A], G[A,F,F], b[A,F])."""
    return _run(_prep_gram(x, u, arm, rows, dt, lib, n_arms, fd, workspace, out, layout,
                           (threshold, alpha, max_iter, unbias)))


def plan_gram(x, u, arm, rows, dt, lib, n_arms=2, fd="smoothed4", workspace=None, out=None,
              layout="patient") -> Plan:
    """``gram`` as a prepared launch (``Plan``); ``plan.out`` = (G, b)."""
    name, args, dev, out, keep = _prep_gram(x, u, arm, rows, dt, lib, n_arms, fd, _plan_ws(workspace), out,
                                            layout)
    return Plan(name, args, dev, out, keep)


def plan_sindy_fit(x, u, arm, rows, dt, lib, threshold, alpha, max_iter=100, unbias=True, n_arms=2,
                   fd="smoothed4", workspace=None, out=None, layout="patient") -> Plan:
    """``sindy_fit`` as a prepared launch; ``plan.out`` = (coef, mask, iters, G, b)."""
    name, args, dev, out, keep = _prep_gram(x, u, arm, rows, dt, lib, n_arms, fd, _plan_ws(workspace), out,
                                            layout, (threshold, alpha, max_iter, unbias))
    return Plan(name, args, dev, out, keep)


def sindy_fit_per_patient(x: torch.Tensor, u: torch.Tensor, arm: torch.Tensor, rows: torch.Tensor, dt: float,
                          lib: PolyLibrary, global_coef: torch.Tensor, threshold: float, alpha: float,
                          max_iter: int = 100, unbias: bool = True, fd: str = "smoothed4",
                          workspace: Workspace | None = None, out: tuple | None = None, layout: str = "patient"):
    """Per-patient refit from the global model's support (insite_sindy_fit_per_patient_f64;
    reference LSQIntialMask per patient, pkpd_simulation.py:791-800).  Returns
    (coef[N, A, F] — the patient's own arm refit, other arms global —, mask[N, F], iters[N])."""
    L = _lib.load()
    N, n_steps, lay = _discovery_inputs(x, u, arm, rows, lib, layout)
    _dev("global_coef", global_coef, torch.float64, 2)
    A, F = global_coef.shape
    if F != lib.n_terms or not global_coef.is_contiguous():
        raise ValueError("global_coef must be a contiguous [n_arms, F] tensor")
    dev = x.device
    if out is None:
        out = (torch.empty((N, A, F), dtype=torch.float64, device=dev),
               torch.empty((N, F), dtype=torch.int8, device=dev),
               torch.empty((N,), dtype=torch.int32, device=dev))
    coef, mask, iters = out
    ws = _ws(workspace, dev, "disc").get(L.insite_per_patient_workspace_bytes(N), dev)
    tab = lib.ctypes_table()
    args = (_p(x), x.stride(0), lay, n_steps, _p(u) if lib.n_statics else ctypes.c_void_p(0), _p(arm), _p(rows), N,
            lib.n_statics, A, tab.ctypes.data_as(ctypes.c_void_p), F, FD_KINDS[fd], float(dt), _p(global_coef),
            float(threshold), float(alpha), int(max_iter), int(bool(unbias)), _p(coef), _p(mask), _p(iters), _p(ws),
            ws.numel())
    return _run(("insite_sindy_fit_per_patient_f64", args, dev, out))


def gram_moments(x: torch.Tensor, u: torch.Tensor, arm: torch.Tensor, rows: torch.Tensor, dt: float,
                 lib: PolyLibrary, threshold: float | None = None, alpha: float = 0.5, max_iter: int = 100,
                 unbias: bool = True, n_arms: int = 2, fd: str = "smoothed4", workspace: Workspace | None = None,
                 out: tuple | None = None, layout: str = "patient"):
    """One pass over x for C4's two fits (insite_gram_moments_f64): the per-arm Gram (G, b) -- plus the global
    STLSQ when ``threshold`` is given (single rank; at N > 1 all-reduce G|b and call ``stlsq``) -- and every
    patient's moments [N, 5] for ``fit_per_patient_moments``.  Returns (coef, mask, iters, G, b, mom) (the
    first three None without threshold)."""
    L = _lib.load()
    N, n_steps, lay = _discovery_inputs(x, u, arm, rows, lib, layout)
    F = lib.n_terms
    dev = x.device
    if out is None:
        out = (torch.empty((n_arms, F), dtype=torch.float64, device=dev) if threshold is not None else None,
               torch.empty((n_arms, F), dtype=torch.int8, device=dev) if threshold is not None else None,
               torch.empty((n_arms,), dtype=torch.int32, device=dev) if threshold is not None else None,
               torch.empty((n_arms, F, F), dtype=torch.float64, device=dev),
               torch.empty((n_arms, F), dtype=torch.float64, device=dev),
               torch.empty((N, 5), dtype=torch.float64, device=dev))
    coef, mask, iters, G, b, mom = out
    ws = _ws(workspace, dev, "disc").get(L.insite_gram_workspace_bytes(N, n_arms, F), dev)
    tab = lib.ctypes_table()
    nul = ctypes.c_void_p(0)
    args = (_p(x), x.stride(0), lay, n_steps, _p(u) if lib.n_statics else nul, _p(arm), _p(rows), N, lib.n_statics,
            n_arms, tab.ctypes.data_as(ctypes.c_void_p), F, FD_KINDS[fd], float(dt),
            float(threshold if threshold is not None else 0.0), float(alpha), int(max_iter), int(bool(unbias)),
            _p(G), _p(b), _p(coef) if coef is not None else nul, _p(mask) if mask is not None else nul,
            _p(iters) if iters is not None else nul, _p(mom), _p(ws), ws.numel())
    return _run(("insite_gram_moments_f64", args, dev, out))


def fit_per_patient_moments(mom: torch.Tensor, u: torch.Tensor, arm: torch.Tensor, rows: torch.Tensor, n_steps: int,
                            lib: PolyLibrary, global_coef: torch.Tensor, threshold: float, alpha: float,
                            max_iter: int = 100, unbias: bool = True, out: tuple | None = None):
    """Per-patient refit from ``gram_moments``' moments (insite_fit_per_patient_moments_f64): the same result
    as ``sindy_fit_per_patient`` without a second pass over x.  Returns (coef[N, A, F], mask[N, F], iters[N])."""
    _dev("mom", mom, torch.float64, 2)
    N = mom.size(0)
    _dev("global_coef", global_coef, torch.float64, 2)
    A, F = global_coef.shape
    if mom.size(1) != 5 or not mom.is_contiguous() or F != lib.n_terms or not global_coef.is_contiguous():
        raise ValueError("mom must be contiguous [N, 5]; global_coef a contiguous [n_arms, F] tensor")
    if arm.numel() != N or rows.numel() != N:
        raise ValueError("arm/rows must have one entry per patient")
    dev = mom.device
    if out is None:
        out = (torch.empty((N, A, F), dtype=torch.float64, device=dev),
               torch.empty((N, F), dtype=torch.int8, device=dev),
               torch.empty((N,), dtype=torch.int32, device=dev))
    coef, mask, iters = out
    tab = lib.ctypes_table()
    args = (_p(mom), _p(u) if lib.n_statics else ctypes.c_void_p(0), _p(arm), _p(rows), N, int(n_steps), lib.n_statics,
            A, tab.ctypes.data_as(ctypes.c_void_p), F, _p(global_coef), float(threshold), float(alpha), int(max_iter),
            int(bool(unbias)), _p(coef), _p(mask), _p(iters))
    return _run(("insite_fit_per_patient_moments_f64", args, dev, out))


def _prep_refit_rollout(mom, u, arm, rows, n_steps, lib, global_coef, threshold, alpha, y0, arm_bits, dt, T, method,
                        max_iter, unbias, drop_below, out, fits):
    _dev("mom", mom, torch.float64, 2)
    N = mom.size(0)
    _dev("global_coef", global_coef, torch.float64, 2)
    A, F = global_coef.shape
    if mom.size(1) != 5 or not mom.is_contiguous() or F != lib.n_terms or not global_coef.is_contiguous():
        raise ValueError("mom must be contiguous [N, 5]; global_coef a contiguous [n_arms, F] tensor")
    _dev("arm", arm, torch.int8, 1)
    _dev("rows", rows, torch.int32, 1)
    _dev("y0", y0, torch.float64, 1)
    if arm.numel() != N or rows.numel() != N or y0.numel() != N:
        raise ValueError("arm/rows/y0 must have one entry per patient")
    if lib.n_statics:
        _dev("u", u, torch.float64, 2)
        if u.size(0) != N or u.size(1) != lib.n_statics or not u.is_contiguous():
            raise ValueError("u must be a contiguous [N, n_statics] tensor")
    ld_bits = _arm_bits_ld(arm_bits, N, T)
    if method not in METHODS:
        raise ValueError(f"method must be one of {sorted(METHODS)}")
    meth, sub = METHODS[method]
    dev = mom.device
    if out is None:
        out = torch.empty((T, N), dtype=torch.float64, device=dev)
    _dev("out", out, torch.float64, 2)
    if out.size(0) < T or out.size(1) < N:
        raise ValueError("out must be [T, >= N]")
    fc, fm, fi = fits if fits is not None else (None, None, None)
    for name, t, dt_, shape in (("fits coef", fc, torch.float64, (N, A, F)), ("fits mask", fm, torch.int8, (N, F)),
                                ("fits iters", fi, torch.int32, (N,))):
        if t is not None:   # the kernel writes these rows: wrong dtype / short tensors would be silent OOB writes
            _dev(name, t, dt_)
            if tuple(t.shape) != shape or not t.is_contiguous() or t.device != dev:
                raise ValueError(f"{name} must be a contiguous {shape} {dt_} tensor on {dev}")
    tab = lib.ctypes_table()
    nul = ctypes.c_void_p(0)
    args = (_p(mom), _p(arm), _p(rows), N, int(n_steps), lib.n_statics, A, tab.ctypes.data_as(ctypes.c_void_p), F,
            _p(global_coef), float(threshold), float(alpha), int(max_iter), int(bool(unbias)), _p(y0),
            _p(u) if lib.n_statics else nul, _p(arm_bits), ld_bits, int(T), float(dt), meth, sub,
            float(drop_below), _p(out), out.stride(0), _p(fc), _p(fm), _p(fi))
    keep = (mom, u, arm, rows, global_coef, y0, arm_bits, out, fc, fm, fi, tab)
    return "insite_refit_rollout_moments_f64", args, dev, out, keep


def refit_rollout_moments(mom: torch.Tensor, u: torch.Tensor, arm: torch.Tensor, rows: torch.Tensor, n_steps: int,
                          lib: PolyLibrary, global_coef: torch.Tensor, threshold: float, alpha: float,
                          y0: torch.Tensor, arm_bits: torch.Tensor, dt: float, T: int, method: str = "euler5",
                          max_iter: int = 100, unbias: bool = True, drop_below: float = 1e-3,
                          out: torch.Tensor | None = None, fits: tuple | None = None):
    """``fit_per_patient_moments`` + the per-patient-coefficient ``rollout`` (TIME_MAJOR_BITS arms) in ONE launch
    (insite_refit_rollout_moments_f64): each lane refits its factual arm's row from its moments in the rollout's
    prologue, so the per-patient coefficient rows never reach HBM.  ``fits`` = (coef[N, A, F], mask[N, F],
    iters[N]) to also receive the refits (any entry None).  Returns y [T, N]."""
    return _run(_prep_refit_rollout(mom, u, arm, rows, n_steps, lib, global_coef, threshold, alpha, y0, arm_bits, dt,
                                    T, method, max_iter, unbias, drop_below, out, fits))


def plan_refit_rollout_moments(mom, u, arm, rows, n_steps, lib, global_coef, threshold, alpha, y0, arm_bits, dt, T,
                               method="euler5", max_iter=100, unbias=True, drop_below=1e-3, out=None, fits=None):
    """``refit_rollout_moments`` prepared once (a ``Plan``)."""
    name, args, dev, out, keep = _prep_refit_rollout(mom, u, arm, rows, n_steps, lib, global_coef, threshold, alpha,
                                                     y0, arm_bits, dt, T, method, max_iter, unbias, drop_below, out,
                                                     fits)
    return Plan(name, args, dev, out, keep)


SEGMENT_FD_KINDS = {"order1": _lib.FD_ORDER1, "smoothed1": _lib.FD_SMOOTHED1}


def _check_segments(x, arm, seq_len, u, lib, n_arms, fd, layout):
    """Validate the F4 (treatment-segment) discovery inputs; returns (N, n_steps)."""
    if layout not in LAYOUTS:
        raise ValueError(f"layout must be one of {sorted(LAYOUTS)}")
    if fd not in SEGMENT_FD_KINDS:
        raise ValueError(f"fd must be one of {sorted(SEGMENT_FD_KINDS)}")
    _dev("x", x, torch.float64, 2)
    _dev("arm", arm, torch.int8, 2)
    _dev("seq_len", seq_len, torch.int32, 1)
    if not 1 <= n_arms <= _lib.MAX_ARMS:
        raise ValueError(f"n_arms must be in [1, {_lib.MAX_ARMS}]")
    N = seq_len.numel()
    if layout == "time":
        n_steps = x.size(0)
        if x.size(1) < N or arm.size(1) < N or arm.size(0) < n_steps - 1:
            raise ValueError("time-major x must be [n_steps, >=N] and arm [>=n_steps-1, >=N]")
    else:
        n_steps = x.size(1)
        if x.size(0) != N or arm.size(0) != N or arm.size(1) < n_steps - 1:
            raise ValueError("patient-major x must be [N, n_steps] and arm [N, >=n_steps-1]")
    if n_steps < 1:
        raise ValueError("need at least one stored sample")
    if lib.n_statics:
        _dev("u", u, torch.float64, 2)
        if u.size(0) != N or u.size(1) != lib.n_statics or u.stride(0) != lib.n_statics:
            raise ValueError("u must be a contiguous [N, n_statics] tensor")
    return N, n_steps


def _prep_segments(x, arm, seq_len, u, dt, lib, n_arms, fd, workspace, out, layout, stlsq_args=None):
    """Validate the F4 (treatment-segment) discovery inputs and pack the C arguments."""
    N, n_steps = _check_segments(x, arm, seq_len, u, lib, n_arms, fd, layout)
    L = _lib.load()
    F = lib.n_terms
    dev = x.device
    ws = _ws(workspace, dev, "disc").get(L.insite_gram_segments_workspace_bytes(N, n_arms, F), dev)
    tab = lib.ctypes_table()
    head = (_p(x), x.stride(0), _p(arm), arm.stride(0), LAYOUTS[layout], n_steps, _p(seq_len),
            _p(u) if lib.n_statics else ctypes.c_void_p(0), N, lib.n_statics, n_arms, tab.ctypes.data_as(ctypes.c_void_p),
            F, SEGMENT_FD_KINDS[fd], float(dt))
    if stlsq_args is None:
        if out is None:
            out = (torch.empty((n_arms, F, F), dtype=torch.float64, device=dev),
                   torch.empty((n_arms, F), dtype=torch.float64, device=dev))
        G, b = out
        return ("insite_gram_segments_f64", head + (_p(G), _p(b), _p(ws), ws.numel()), dev, out,
                (x, arm, seq_len, u, tab, ws, *out))
    threshold, alpha, max_iter, unbias = stlsq_args
    if out is None:
        out = (torch.empty((n_arms, F), dtype=torch.float64, device=dev),
               torch.empty((n_arms, F), dtype=torch.int8, device=dev),
               torch.empty((n_arms,), dtype=torch.int32, device=dev),
               torch.empty((n_arms, F, F), dtype=torch.float64, device=dev),
               torch.empty((n_arms, F), dtype=torch.float64, device=dev))
    coef, mask, iters, G, b = out
    args = head + (float(threshold), float(alpha), int(max_iter), int(bool(unbias)), _p(G), _p(b), _p(coef), _p(mask),
                   _p(iters), _p(ws), ws.numel())
    return "insite_sindy_fit_segments_f64", args, dev, out, (x, arm, seq_len, u, tab, ws, *out)


def gram_segments(x: torch.Tensor, arm: torch.Tensor, seq_len: torch.Tensor, u: torch.Tensor, dt: float,
                  lib: PolyLibrary, n_arms: int = 4, fd: str = "order1", workspace: Workspace | None = None,
                  out: tuple | None = None, layout: str = "patient"):
    """Per-arm Gram of the treatment-segment regression (insite_gram_segments_f64; reference
    process_sindy_training_data, pkpd/utils.py:433-462).  layout "patient": x [N, T], arm [N, >=T-1]
    (the reference's arrays, arm = argmax of the one-hot); "time": x [T, >=N], arm [>=T-1, >=N].
    Returns (G[A,F,F], b[A,F]); G[a,0,0] is arm a's sample count."""
    return _run(_prep_segments(x, arm, seq_len, u, dt, lib, n_arms, fd, workspace, out, layout))


def sindy_fit_segments(x: torch.Tensor, arm: torch.Tensor, seq_len: torch.Tensor, u: torch.Tensor, dt: float,
                       lib: PolyLibrary, threshold: float, alpha: float, max_iter: int = 100, unbias: bool = True,
                       n_arms: int = 4, fd: str = "order1", workspace: Workspace | None = None,
                       out: tuple | None = None, layout: str = "patient"):
    """cancer_sim / EQ_5 discovery in two launches (insite_sindy_fit_segments_f64): the segment-split
    Gram kernel, then the fixed-order reduction fused with one STLSQ per arm — replaces the four
    ``SINDy(FiniteDifference(order=1)).fit`` calls (reference sindy.py:193-216).
    Returns (coef[A,F], mask[A,F], iters[A], G[A,F,F], b[A,F])."""
    return _run(_prep_segments(x, arm, seq_len, u, dt, lib, n_arms, fd, workspace, out, layout,
                               (threshold, alpha, max_iter, unbias)))


def gen_gram_segments(x: torch.Tensor, arm: torch.Tensor, seq_len: torch.Tensor, u: torch.Tensor, dt: float,
                      lib: PolyLibrary, n_arms: int = 4, fd: str = "order1", workspace: Workspace | None = None,
                      out: tuple | None = None, layout: str = "patient"):
    """Per-arm Gram of the treatment-segment regression with a GENERAL library (state exponents <= 4: the
    degree-4 ablation on cancer_sim / EQ_5, sindy.py:185-186; insite_gen_gram_segments_f64).  Arrays as
    ``gram_segments``.  Returns (G [A, F, F], b [A, F])."""
    N, n_steps = _check_segments(x, arm, seq_len, u, lib, n_arms, fd, layout)
    L = _lib.load()
    F = lib.n_terms
    dev = x.device
    ws = _ws(workspace, dev, "scratch").get(L.insite_gen_gram_segments_workspace_bytes(N, n_arms, F), dev)
    if out is None:
        out = (torch.empty((n_arms, F, F), dtype=torch.float64, device=dev),
               torch.empty((n_arms, F), dtype=torch.float64, device=dev))
    G, b = out
    tab = lib.ctypes_table()
    args = (_p(x), x.stride(0), _p(arm), arm.stride(0), LAYOUTS[layout], n_steps, _p(seq_len),
            _p(u) if lib.n_statics else ctypes.c_void_p(0), lib.n_statics, N, n_arms,
            tab.ctypes.data_as(ctypes.c_void_p), F, SEGMENT_FD_KINDS[fd], float(dt), _p(G), _p(b), _p(ws), ws.numel())
    return _run(("insite_gen_gram_segments_f64", args, dev, out))


def plan_gram_segments(x, arm, seq_len, u, dt, lib, n_arms=4, fd="order1", workspace=None, out=None,
                       layout="patient") -> Plan:
    """``gram_segments`` as a prepared launch; ``plan.out`` = (G, b)."""
    name, args, dev, out, keep = _prep_segments(x, arm, seq_len, u, dt, lib, n_arms, fd, _plan_ws(workspace),
                                                out, layout)
    return Plan(name, args, dev, out, keep)


def plan_sindy_fit_segments(x, arm, seq_len, u, dt, lib, threshold, alpha, max_iter=100, unbias=True, n_arms=4,
                            fd="order1", workspace=None, out=None, layout="patient") -> Plan:
    """``sindy_fit_segments`` as a prepared launch; ``plan.out`` = (coef, mask, iters, G, b)."""
    name, args, dev, out, keep = _prep_segments(x, arm, seq_len, u, dt, lib, n_arms, fd, _plan_ws(workspace),
                                                out, layout, (threshold, alpha, max_iter, unbias))
    return Plan(name, args, dev, out, keep)


GEN_FD_KINDS = {"smoothed4": _lib.FD_SMOOTHED4, "order4": _lib.FD_ORDER4, "order1": _lib.FD_ORDER1,
                "smoothed1": _lib.FD_SMOOTHED1}


def gen_gram(x: torch.Tensor, u: torch.Tensor | None, rows: torch.Tensor, dt: float, lib: PolyLibrary,
             group: torch.Tensor | None = None, n_groups: int = 1, step_in: torch.Tensor | None = None,
             fd: str = "smoothed4", layout: str = "patient", workspace: Workspace | None = None,
             out: tuple | None = None):
    """General one-state Gram (insite_gen_gram_f64): libraries with state exponents up to 4 (the degree-4
    ablation, reference sindy.py:185-186) and/or ``lib.n_inputs`` per-step binary inputs (the joint model,
    pkpd/utils.py:486-497).  x [N, T] ("patient") or [T, >=N] ("time") f64; step_in int8 in the same
    layout, bit i = input i; group [N] int8 (regression of each patient, e.g. its arm; None = one
    regression); rows [N] int32.  Returns (G [n_groups, F, F], b [n_groups, F])."""
    if layout not in LAYOUTS:
        raise ValueError(f"layout must be one of {sorted(LAYOUTS)}")
    if fd not in GEN_FD_KINDS:
        raise ValueError(f"fd must be one of {sorted(GEN_FD_KINDS)}")
    _dev("x", x, torch.float64, 2)
    _dev("rows", rows, torch.int32, 1)
    N = rows.numel()
    n_steps = x.size(0) if layout == "time" else x.size(1)
    if (x.size(1) < N) if layout == "time" else (x.size(0) != N):
        raise ValueError("x must hold one series per patient ([T, >=N] time-major, [N, T] patient-major)")
    if group is not None:
        _dev("group", group, torch.int8, 1)
        if group.numel() != N:
            raise ValueError("group must have one entry per patient")
    if not 1 <= n_groups <= _lib.MAX_ARMS:
        raise ValueError(f"n_groups must be in [1, {_lib.MAX_ARMS}]")
    U = lib.n_statics
    if U:
        _dev("u", u, torch.float64, 2)
        if u.size(0) != N or u.size(1) != U or u.stride(0) != U:
            raise ValueError("u must be a contiguous [N, n_statics] tensor")
    if lib.n_inputs:
        _dev("step_in", step_in, torch.int8, 2)
        if (step_in.size(1) < N or step_in.size(0) < n_steps) if layout == "time" else \
                (step_in.size(0) != N or step_in.size(1) < n_steps):
            raise ValueError("step_in must cover every (patient, step) of x")
    L = _lib.load()
    F = lib.n_terms
    dev = x.device
    ws = _ws(workspace, dev, "scratch").get(L.insite_gen_gram_workspace_bytes(N, n_steps, n_groups, F), dev)
    if out is None:
        out = (torch.empty((n_groups, F, F), dtype=torch.float64, device=dev),
               torch.empty((n_groups, F), dtype=torch.float64, device=dev))
    G, b = out
    tab = lib.ctypes_table()
    args = (_p(x), x.stride(0), LAYOUTS[layout], n_steps, _p(u) if U else ctypes.c_void_p(0), U,
            _p(step_in) if lib.n_inputs else ctypes.c_void_p(0), step_in.stride(0) if lib.n_inputs else 0,
            lib.n_inputs, _p(group), n_groups, _p(rows), N, tab.ctypes.data_as(ctypes.c_void_p), F, GEN_FD_KINDS[fd],
            float(dt), _p(G), _p(b), _p(ws), ws.numel())
    return _run(("insite_gen_gram_f64", args, dev, out))


def gen_sindy_fit(x, u, rows, dt, lib, threshold, alpha, group=None, n_groups=1, step_in=None, fd="smoothed4",
                  layout="patient", max_iter=100, unbias=True, workspace=None):
    """``gen_gram`` then the batched STLSQ (insite_stlsq_f64; F > 9 runs one wavefront per system).
    Returns (coef [n_groups, F], mask, iters, G, b)."""
    G, b = gen_gram(x, u, rows, dt, lib, group, n_groups, step_in, fd, layout, workspace)
    coef, mask, iters = stlsq(G, b, threshold, alpha, max_iter, unbias)
    return coef, mask, iters, G, b


def _prep_stlsq(G, b, threshold, alpha, max_iter, unbias, out):
    _dev("G", G, torch.float64)
    _dev("b", b, torch.float64)
    F = G.shape[-1]
    S = G.numel() // (F * F)
    if b.numel() != S * F or not G.is_contiguous() or not b.is_contiguous():
        raise ValueError("G/b must be contiguous [S,F,F] / [S,F]")
    if out is None:
        out = (torch.empty((S, F), dtype=torch.float64, device=G.device),
               torch.empty((S, F), dtype=torch.int8, device=G.device),
               torch.empty((S,), dtype=torch.int32, device=G.device))
    coef, mask, iters = out
    args = (_p(G), _p(b), S, F, float(threshold), float(alpha), int(max_iter), int(bool(unbias)), _p(coef), _p(mask),
            _p(iters))
    return "insite_stlsq_f64", args, G.device, out, (G, b, *out)


def stlsq(G: torch.Tensor, b: torch.Tensor, threshold: float, alpha: float, max_iter: int = 100,
          unbias: bool = True, out: tuple | None = None):
    """Batched STLSQ on Gram systems (insite_stlsq_f64).  G [S,F,F], b [S,F]."""
    return _run(_prep_stlsq(G, b, threshold, alpha, max_iter, unbias, out))


def plan_stlsq(G, b, threshold, alpha, max_iter=100, unbias=True, out=None) -> Plan:
    name, args, dev, out, keep = _prep_stlsq(G, b, threshold, alpha, max_iter, unbias, out)
    return Plan(name, args, dev, out, keep)


def _prep_rollout(y0, u, arm, coef, lib, dt, method, substeps, drop_below, T, out, layout):
    if layout not in ROLLOUT_LAYOUTS:
        raise ValueError(f"layout must be one of {sorted(ROLLOUT_LAYOUTS)}")
    tm = layout != "patient"
    _dev("y0", y0, torch.float64, 1)
    N = y0.numel()
    ld_arm = None
    if layout == "time_bits":   # time-major [>= T, >= ceil(N/32)] or tile-major [ceil(N/64), >= T, 2] int32 words
        if not isinstance(arm, torch.Tensor) or arm.dim() not in (2, 3):
            raise ValueError("bit-packed arm must be [>=T, >=ceil(N/32)] (or tile-major [ceil(N/64), >=T, 2]) int32")
        T = (arm.size(0) if arm.dim() == 2 else arm.size(1)) if T is None else int(T)
        ld_arm = _arm_bits_ld(arm, N, T)
    elif tm:
        _dev("arm", arm, torch.int8, 2)
        T = arm.size(0) if T is None else int(T)
        if arm.size(1) < N or arm.size(0) < T:
            raise ValueError("time-major arm must be [>=T, >=N]")
    else:
        _dev("arm", arm, torch.int8, 2)
        T = arm.size(1) if T is None else int(T)
        if arm.size(0) != N or arm.size(1) < T:
            raise ValueError("arm must be [N, >=T]")
    if lib.n_statics:
        _dev("u", u, torch.float64, 2)
        if u.size(0) != N or u.size(1) != lib.n_statics or u.stride(0) != lib.n_statics:
            raise ValueError("u must be a contiguous [N, n_statics] tensor")
    _dev("coef", coef, torch.float64)
    if not coef.is_contiguous():
        raise ValueError("coef must be contiguous")
    F = lib.n_terms
    if coef.dim() == 2:
        A = coef.size(0)
        stride = 0
    elif coef.dim() == 3:
        if coef.size(0) != N:
            raise ValueError("per-patient coef must be [N, A, F]")
        A = coef.size(1)
        stride = A * F
    else:
        raise ValueError("coef must be [A,F] or [N,A,F]")
    if coef.size(-1) != F:
        raise ValueError("coef last dim must equal the library size")
    m, default_sub = METHODS[method]
    sub = int(substeps or default_sub)
    shape = (T, N) if tm else (N, T)
    if out is None:
        out = torch.empty(shape, dtype=torch.float64, device=y0.device)
    else:
        _dev("out", out, torch.float64, 2)
        if out.size(0) != shape[0] or out.size(1) < shape[1]:
            raise ValueError(f"out must be {shape}")
    tab = lib.ctypes_table()
    args = (_p(y0), _p(u) if lib.n_statics else ctypes.c_void_p(0), _p(arm),
            arm.stride(0) if ld_arm is None else ld_arm, _p(coef), stride,
            tab.ctypes.data_as(ctypes.c_void_p), F, N, T, lib.n_statics, A, float(dt), m, sub, float(drop_below),
            _p(out), out.stride(0), ROLLOUT_LAYOUTS[layout])
    return "insite_rollout_f64", args, y0.device, out, (y0, u, arm, coef, tab, out)


def rollout(y0: torch.Tensor, u: torch.Tensor, arm: torch.Tensor, coef: torch.Tensor, lib: PolyLibrary,
            dt: float, method: str = "euler5", substeps: int | None = None, drop_below: float = 1e-3,
            T: int | None = None, out: torch.Tensor | None = None, layout: str = "patient"):
    """Batched open-loop rollout (insite_rollout_f64).

    y0 [N] f64, u [N,U] f64, coef [A,F] (global model) or [N,A,F] (per-patient).
    layout "patient":   arm int8 [N, >=T], returns y [N,T] (the reference's [N, T] arrays).
    layout "time":      arm int8 [T, >=N], returns y [T,N] (one contiguous run per step).
    layout "time_bits": arm int32 [T, >=ceil(N/32)] bitmask (pack_arm_bits; A <= 2), y [T,N] —
                        the fast layout on MI355X; or the same bits tile-major,
                        int32 [ceil(N/64), >=T, 2] (tile_major_bits).  Row k of y is the state
                        after observation interval k."""
    return _run(_prep_rollout(y0, u, arm, coef, lib, dt, method, substeps, drop_below, T, out, layout))


def plan_rollout(y0, u, arm, coef, lib, dt, method="euler5", substeps=None, drop_below=1e-3, T=None, out=None,
                 layout="patient") -> Plan:
    """``rollout`` as a prepared launch; ``plan.out`` = y."""
    name, args, dev, out, keep = _prep_rollout(y0, u, arm, coef, lib, dt, method, substeps, drop_below, T, out, layout)
    return Plan(name, args, dev, out, keep)


def _prep_fit_rollout(x, u, arm, rows, dt, lib, threshold, alpha, max_iter, unbias, fd, workspace, out,
                      y0, ru, arm_bits, coef_in, rdt, method, substeps, drop_below, T, y_out, gram_blocks):
    gname, gargs, dev, gout, gkeep = _prep_gram(x, u, arm, rows, dt, lib, 2, fd, workspace, out, "time",
                                               (threshold, alpha, max_iter, unbias))
    rname, rargs, rdev, y_out, rkeep = _prep_rollout(y0, ru, arm_bits, coef_in, lib, rdt, method, substeps,
                                                     drop_below, T, y_out, "time_bits")
    if rdev != dev:
        raise ValueError("both cohorts must live on one device")
    if coef_in.dim() != 2 or coef_in.size(0) != 2:
        raise ValueError("coef_in must be a contiguous [2, F] global model")
    # insite_sindy_fit_f64 args: x ldx layout n_steps u arm rows N U A tab F fd dt thr alpha it unbias G b coef mask
    # iters ws wsb;  insite_rollout_f64 args: y0 u arm lda coef stride tab F N T U A dt method sub drop y ldy layout
    g, r = gargs, rargs
    args = (g[0], g[1], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10], g[11], g[12], g[13], g[14], g[15], g[16],
            g[17], g[18], g[19], g[20], g[21], g[22],
            r[0], r[1], r[2], r[3], r[4], r[8], r[9], r[12], r[13], r[14], r[15], r[16], r[17],
            int(gram_blocks), g[23], g[24])
    return "insite_fit_rollout_f64", args, dev, (gout, y_out), gkeep + rkeep


def fit_rollout(x, u, arm, rows, dt, lib, threshold, alpha, y0, ru, arm_bits, coef_in, rdt, method="rk4",
                max_iter=100, unbias=True, fd="smoothed4", substeps=None, drop_below=1e-3, T=None, workspace=None,
                out=None, y_out=None, gram_blocks=0):
    """Fused step (insite_fit_rollout_f64): in ONE launch, the discovery of cohort (x [T, >=N]
    time-major, u, arm, rows) -- ``sindy_fit`` with 2 arms and the 7-term library -- and the rollout
    of another cohort (y0, ru, arm_bits [T, >=ceil(N/32)] int32) with the known global model coef_in
    [2, F] -- ``rollout(layout="time_bits")``.  Returns ((coef, mask, iters, G, b), y)."""
    return _run(_prep_fit_rollout(x, u, arm, rows, dt, lib, threshold, alpha, max_iter, unbias, fd, workspace, out,
                                  y0, ru, arm_bits, coef_in, rdt, method, substeps, drop_below, T, y_out,
                                  gram_blocks))


def plan_fit_rollout(x, u, arm, rows, dt, lib, threshold, alpha, y0, ru, arm_bits, coef_in, rdt, method="rk4",
                     max_iter=100, unbias=True, fd="smoothed4", substeps=None, drop_below=1e-3, T=None,
                     workspace=None, out=None, y_out=None, gram_blocks=0) -> Plan:
    """``fit_rollout`` as a prepared launch; ``plan.out`` = ((coef, mask, iters, G, b), y)."""
    name, args, dev, out, keep = _prep_fit_rollout(x, u, arm, rows, dt, lib, threshold, alpha, max_iter, unbias, fd,
                                                   _plan_ws(workspace), out, y0, ru, arm_bits, coef_in, rdt,
                                                   method, substeps, drop_below, T, y_out, gram_blocks)
    return Plan(name, args, dev, out, keep)


def _prep_fit_rollout_deferred(x, u, arm, rows, dt, lib, threshold, alpha, max_iter, unbias, fd, workspace, out,
                               y0, ru, arm_bits, coef_in, rdt, method, substeps, drop_below, T, y_out, gram_blocks,
                               slot, finalize_prev):
    if workspace is None:
        raise ValueError("the deferred step keeps its partial slots between calls: pass the stream's Workspace")
    if slot not in (0, 1):
        raise ValueError("slot must be 0 or 1")
    name, args, dev, outs, keep = _prep_fit_rollout(x, u, arm, rows, dt, lib, threshold, alpha, max_iter, unbias, fd,
                                                    False, out, y0, ru, arm_bits, coef_in, rdt, method, substeps,
                                                    drop_below, T, y_out, gram_blocks)
    nbytes = _lib.load().insite_fit_rollout_deferred_workspace_bytes(int(args[6]), 2, lib.n_terms)
    ws = workspace.claim("deferred").get(nbytes, dev)
    args = args[:-2] + (int(slot), int(bool(finalize_prev)), _p(ws), ws.numel())
    return "insite_fit_rollout_deferred_f64", args, dev, outs, keep + (ws,)


def fit_rollout_deferred(x, u, arm, rows, dt, lib, threshold, alpha, y0, ru, arm_bits, coef_in, rdt, slot,
                         finalize_prev, workspace, method="rk4", max_iter=100, unbias=True, fd="smoothed4",
                         substeps=None, drop_below=1e-3, T=None, out=None, y_out=None, gram_blocks=0):
    """The fused step with the discovery's finalisation deferred by one call (insite_fit_rollout_deferred_f64):
    streams the Gram of cohort (x, u, arm, rows) into partial slot ``slot`` of ``workspace`` (a Workspace kept
    for the whole stream of calls), and -- with ``finalize_prev`` -- reduces the other slot (the previous
    call's cohort) into ``out`` = (coef, mask, iters, G, b), all in the launch that rolls out (y0, ru,
    arm_bits) with coef_in.  Returns ((coef, mask, iters, G, b), y); the first tuple holds the PREVIOUS
    call's cohort (untouched without ``finalize_prev``)."""
    return _run(_prep_fit_rollout_deferred(x, u, arm, rows, dt, lib, threshold, alpha, max_iter, unbias, fd,
                                           workspace, out, y0, ru, arm_bits, coef_in, rdt, method, substeps,
                                           drop_below, T, y_out, gram_blocks, slot, finalize_prev))


def plan_fit_rollout_deferred(x, u, arm, rows, dt, lib, threshold, alpha, y0, ru, arm_bits, coef_in, rdt, slot,
                              finalize_prev, workspace, method="rk4", max_iter=100, unbias=True, fd="smoothed4",
                              substeps=None, drop_below=1e-3, T=None, out=None, y_out=None, gram_blocks=0) -> Plan:
    """``fit_rollout_deferred`` as a prepared launch."""
    return Plan(*_prep_fit_rollout_deferred(x, u, arm, rows, dt, lib, threshold, alpha, max_iter, unbias, fd,
                                            workspace, out, y0, ru, arm_bits, coef_in, rdt, method, substeps,
                                            drop_below, T, y_out, gram_blocks, slot, finalize_prev))


def _prep_fit_rollout_lagged(x, u, arm, rows, dt, lib, threshold, alpha, max_iter, unbias, fd, workspace, red,
                             fit_in, fit_out, y0, ru, arm_bits, coef_in, rdt, method, substeps, drop_below, T, y_out,
                             gram_blocks, slot, reduce_prev):
    if workspace is None:
        raise ValueError("the lagged step keeps its partial slots between calls: pass the stream's Workspace")
    if slot not in (0, 1):
        raise ValueError("slot must be 0 or 1")
    F = lib.n_terms
    dev = x.device
    G, b = red
    for name, t, shape in (("G_out", G, (2, F, F)), ("b_out", b, (2, F))):
        _dev(name, t, torch.float64)
        if tuple(t.shape) != shape or not t.is_contiguous():
            raise ValueError(f"{name} must be a contiguous {shape} f64 tensor")
    Gf, bf = fit_in if fit_in is not None else (None, None)
    if fit_in is not None:
        for name, t, shape in (("G_fit", Gf, (2, F, F)), ("b_fit", bf, (2, F))):
            _dev(name, t, torch.float64)
            if tuple(t.shape) != shape or not t.is_contiguous():
                raise ValueError(f"{name} must be a contiguous {shape} f64 tensor")
        if Gf.data_ptr() == G.data_ptr() or bf.data_ptr() == b.data_ptr():
            raise ValueError("G_fit / b_fit must not alias this call's G_out / b_out")
        if fit_out is None:
            raise ValueError("fit_out = (coef, mask, iters) receives the solve of G_fit / b_fit")
    coef, mask, iters = fit_out if fit_out is not None else (None, None, None)
    # the deferred packing (validation of both halves), then the lagged argument order
    name, args, dev, outs, keep = _prep_fit_rollout(x, u, arm, rows, dt, lib, threshold, alpha, max_iter, unbias, fd,
                                                    False, (coef if coef is not None else torch.empty(
                                                        (2, F), dtype=torch.float64, device=dev),
                                                        mask if mask is not None else torch.empty(
                                                            (2, F), dtype=torch.int8, device=dev),
                                                        iters if iters is not None else torch.empty(
                                                            (2,), dtype=torch.int32, device=dev), G, b),
                                                    y0, ru, arm_bits, coef_in, rdt, method, substeps, drop_below, T,
                                                    y_out, gram_blocks)
    nbytes = _lib.load().insite_fit_rollout_deferred_workspace_bytes(int(args[6]), 2, F)
    ws = workspace.claim("deferred").get(nbytes, dev)
    nul = ctypes.c_void_p(0)
    # fit_rollout args: [0..16] discovery head, 17 G, 18 b, 19 coef, 20 mask, 21 iters, 22.. rollout, -3 gram_blocks
    args = (args[:19] + (_p(Gf) if Gf is not None else nul, _p(bf) if bf is not None else nul)
            + (_p(coef) if coef is not None else nul, _p(mask) if mask is not None else nul,
               _p(iters) if iters is not None else nul)
            + args[22:-2] + (int(slot), int(bool(reduce_prev)), _p(ws), ws.numel()))
    return "insite_fit_rollout_lagged_f64", args, dev, (red, fit_out, outs[1]), keep + (ws, Gf, bf)


def plan_fit_rollout_lagged(x, u, arm, rows, dt, lib, threshold, alpha, y0, ru, arm_bits, coef_in, rdt, slot,
                            reduce_prev, workspace, red, fit_in=None, fit_out=None, method="rk4", max_iter=100,
                            unbias=True, fd="smoothed4", substeps=None, drop_below=1e-3, T=None, y_out=None,
                            gram_blocks=0) -> Plan:
    """The N > 1 form of the deferred step (insite_fit_rollout_lagged_f64): streams cohort (x, u, arm, rows) into
    slot ``slot``; with ``reduce_prev`` reduces the other slot into this rank's ``red`` = (G, b) (no STLSQ: the
    ranks all-reduce it between calls); with ``fit_in`` = (G, b) (an all-reduced system) solves its STLSQ into
    ``fit_out`` = (coef, mask, iters); rolls out (y0, ru, arm_bits) with ``coef_in``.  ``plan.out`` =
    (red, fit_out, y)."""
    return Plan(*_prep_fit_rollout_lagged(x, u, arm, rows, dt, lib, threshold, alpha, max_iter, unbias, fd, workspace,
                                          red, fit_in, fit_out, y0, ru, arm_bits, coef_in, rdt, method, substeps,
                                          drop_below, T, y_out, gram_blocks, slot, reduce_prev))


RK45_ATTEMPT_BINS = 1024   # the counting sort's bin count (kRkBinMax): attempt counts above 1022 share the last bin


def rk45_order(n_obs: torch.Tensor, T_max: int, out: torch.Tensor | None = None) -> torch.Tensor:
    """Lane order for ``rollout_rk45``: rows sorted by n_obs, descending (insite_rk45_order_i32, a
    counting sort on the device).  Scheduling only: the rollout's outputs do not depend on it."""
    _dev("n_obs", n_obs, torch.int32, 1)
    N = n_obs.numel()
    if out is None:
        out = torch.empty((N,), dtype=torch.int32, device=n_obs.device)
    nb = _lib.load().insite_rk45_order_workspace_bytes(int(T_max))
    # a workspace of its own: the counting sort's totals / cursors reset themselves at the end of every call, so the
    # buffer must be zero at its first use and hold nothing else (insite_hip.h)
    ws = _default_ws(n_obs.device, "order").get(nb, n_obs.device)
    args = (_p(n_obs), N, int(T_max), _p(out), _p(ws), ws.numel())
    return _run(("insite_rk45_order_i32", args, n_obs.device, out))


def _rk45_prep(y0, u, arm_bits, t_obs, n_obs, coef, lib, rtol, atol, drop_below, out, steps, order, layout,
               plan):
    """rollout_rk45's validation and argument packing; plan=True returns the packed calls (plan_rollout_rk45)."""
    if layout not in ("time", "patient"):
        raise ValueError("layout must be 'time' or 'patient'")
    pm = layout == "patient"
    _dev("y0", y0, torch.float64, 1)
    N = y0.numel()
    _dev("t_obs", t_obs, torch.float64, 2)
    Tm = t_obs.size(1) if pm else t_obs.size(0)
    if (t_obs.size(0) if pm else t_obs.size(1)) < N or (pm and t_obs.size(0) != N):
        raise ValueError("t_obs must be [N, T_max]" if pm else "t_obs must be [T_max, >=N]")
    _dev("arm_bits", arm_bits, torch.int32, 2)
    if pm:
        if arm_bits.size(0) != N or arm_bits.size(1) < max(1, (Tm - 1 + 31) // 32):
            raise ValueError("arm_bits must be [N, >=ceil((T_max-1)/32)] int32")
    elif arm_bits.size(0) < Tm or arm_bits.size(1) < (N + 31) // 32:
        raise ValueError("arm_bits must be [>=T_max, >=ceil(N/32)] int32")
    _dev("n_obs", n_obs, torch.int32, 1)
    if n_obs.numel() != N:
        raise ValueError("n_obs must have one entry per patient")
    if lib.n_statics:
        _dev("u", u, torch.float64, 2)
        if u.size(0) != N or u.size(1) != lib.n_statics or u.stride(0) != lib.n_statics:
            raise ValueError("u must be a contiguous [N, n_statics] tensor")
    _dev("coef", coef, torch.float64)
    F = lib.n_terms
    if coef.dim() == 2:
        A, stride = coef.size(0), 0
    elif coef.dim() == 3 and coef.size(0) == N:
        A, stride = coef.size(1), coef.size(1) * F
    else:
        raise ValueError("coef must be [A,F] or [N,A,F]")
    if coef.size(-1) != F or not coef.is_contiguous():
        raise ValueError("coef must be contiguous with the library's F columns")
    shape = (N, Tm) if pm else (Tm, N)
    if out is None:
        out = torch.full(shape, float("nan"), dtype=torch.float64, device=y0.device)
    else:
        _dev("out", out, torch.float64, 2)
        if out.size(0) < shape[0] or out.size(1) < shape[1] or (pm and out.size(0) != N):
            raise ValueError(f"out must be {'[N, >=T_max]' if pm else '[T_max, >=N]'}")
    # the binning key: n_obs (order=True), or -- order="attempts" -- the per-patient attempt counts the previous call
    # left in ``steps`` (a re-rolled cohort takes the same counts again, so its waves group equal attempt counts: wave
    # divergence 1.07 -> ~1.01 at C5's shape); the first call bins whatever ``steps`` holds (zeros when allocated here)
    key, key_T = n_obs, int(Tm)
    if isinstance(order, str):
        if order != "attempts":
            raise ValueError("order must be True, False/None, 'attempts' or a [N] int32 permutation")
        if steps is None:
            steps = torch.zeros((N,), dtype=torch.int32, device=y0.device)
        _dev("steps", steps, torch.int32, 1)
        key, key_T, order = steps, RK45_ATTEMPT_BINS - 1, True
    if steps is None:
        steps = torch.empty((N,), dtype=torch.int32, device=y0.device)
    order_call = None
    if order is True:
        if plan:   # the plan bins into its own buffer with its own workspace, per call
            order = torch.empty((N,), dtype=torch.int32, device=n_obs.device)
            wsb = _lib.load().insite_rk45_order_workspace_bytes(key_T)
            ows = torch.zeros((max(1, (wsb + 7) // 8),), dtype=torch.float64, device=n_obs.device)
            order_call = ("insite_rk45_order_i32", (_p(key), N, key_T, _p(order), _p(ows), wsb), (order, ows, key))
        else:
            order = rk45_order(key, key_T)
    elif order is False:
        order = None
    elif order is not None:
        _dev("order", order, torch.int32, 1)
        if order.numel() != N:
            raise ValueError("order must be a [N] int32 permutation")
    tab = lib.ctypes_table()
    args = (_p(y0), _p(u) if lib.n_statics else ctypes.c_void_p(0), _p(arm_bits), arm_bits.stride(0), _p(t_obs),
            t_obs.stride(0), _p(n_obs), _p(coef), stride, tab.ctypes.data_as(ctypes.c_void_p), F, N, Tm,
            lib.n_statics, A, float(rtol), float(atol), float(drop_below), _p(out), out.stride(0), _p(steps),
            _p(order), _lib.LAYOUT_PATIENT_MAJOR_BITS if pm else _lib.LAYOUT_TIME_MAJOR_BITS)
    if plan:
        keep = (y0, u, arm_bits, t_obs, n_obs, coef, tab, out, steps, order)
        return order_call, ("insite_rollout_rk45_f64", args, keep), (out, steps)
    return _run(("insite_rollout_rk45_f64", args, y0.device, (out, steps)))


def rollout_rk45(y0: torch.Tensor, u: torch.Tensor, arm_bits: torch.Tensor, t_obs: torch.Tensor,
                 n_obs: torch.Tensor, coef: torch.Tensor, lib: PolyLibrary, rtol: float = 1.4e-8, atol: float = 1.4e-8,
                 drop_below: float = 1e-3, out: torch.Tensor | None = None, steps: torch.Tensor | None = None,
                 order: torch.Tensor | bool | None = True, layout: str = "time"):
    """Adaptive RK45 rollout on per-patient irregular observation grids (insite_rollout_rk45_f64;
    configuration C5).  y0 [N] f64, u [N,U] f64, n_obs [N] int32, coef [A,F] or [N,A,F].
    layout "time":    t_obs [T_max, >=N] f64, arm_bits [T_max, >=ceil(N/32)] int32 (pack_arm_bits of the
                      time-major arms), y [T_max, N] (row k = state at t_obs[k + 1]);
    layout "patient": t_obs [N, >=T_max] f64, arm_bits [N, >=ceil((T_max-1)/32)] int32 (pack_arm_bits of
                      the patient-major arms [N, T]), y [N, T_max] -- the fast layout.
    ``order``: True bins the rows by n_obs on the device first (``rk45_order``, part of the call), "attempts" by
    the attempt counts a previous call left in ``steps``, a [N] int32 permutation is used as given, None/False runs
    lane r on row r.  Outputs do not depend on it.
    Returns (y, step attempts [N] int32); y elements past a patient's grid are left as they were (NaN
    when ``out`` is None)."""
    return _rk45_prep(y0, u, arm_bits, t_obs, n_obs, coef, lib, rtol, atol, drop_below, out, steps, order, layout,
                      False)


class Rk45Plan:
    """``rollout_rk45`` prepared once (inputs validated, buffers and arguments packed): a call enqueues the n_obs
    counting sort into the plan's own order buffer (when binning) and the RK45 rollout -- two C calls, no host
    work beyond them.  ``out`` = (y, step attempts), bitwise those of ``rollout_rk45``.  The plan keeps references
    to its inputs: refresh them in place between calls or make a new plan."""

    def __init__(self, calls, device, out):
        L = _lib.load()
        self._calls = [(getattr(L, name), args) for name, args, _ in calls]
        self._keep = tuple(k for _, _, k in calls)
        self.device = torch.device(device)
        self.out = out

    def __call__(self, stream: torch.cuda.Stream | None = None):
        h = ctypes.c_void_p((stream if stream is not None else torch.cuda.current_stream(self.device)).cuda_stream)
        for fn, args in self._calls:
            st = fn(*args, h)
            if st:
                _lib.check(getattr(fn, "__name__", "rk45 plan"), st)
        return self.out


def plan_rollout_rk45(y0, u, arm_bits, t_obs, n_obs, coef, lib, rtol=1.4e-8, atol=1.4e-8, drop_below=1e-3, out=None,
                      steps=None, order=True, layout="time") -> Rk45Plan:
    """``rollout_rk45`` as a plan (the C5 bench's per-step call): the same validation, done once."""
    order_call, call, outs = _rk45_prep(y0, u, arm_bits, t_obs, n_obs, coef, lib, rtol, atol, drop_below, out, steps,
                                        order, layout, True)
    return Rk45Plan(([order_call] if order_call else []) + [call], y0.device, outs)


def refine_terms(lib: PolyLibrary, n_coef_rows: int):
    """Per-coefficient description of a global model for ``insite_refine_general_f64``: (arm mask int32
    [n_coef], exponents int8 [n_coef, 1 + n_statics], number of arms).  Per-arm models (lib.n_inputs = 0):
    coefficient (a, j) acts on arm a.  The joint model (lib.n_inputs > 0, one coefficient row): the arm of
    a step is its treatment bit code and column j acts on every code that switches its treatment inputs
    on (binary inputs: their exponents drop out) -- the fold of ``SINDY._fold_joint``."""
    e = lib.exps.astype(np.int64)
    n_in, U, F = lib.n_inputs, lib.n_statics, lib.n_terms
    keep = [0] + list(range(1 + n_in, 1 + n_in + U))
    if n_in == 0:
        A = n_coef_rows
        mask = np.array([1 << a for a in range(A) for _ in range(F)], dtype=np.int32)
        exps = np.tile(e[:, keep], (A, 1))
    else:
        if n_coef_rows != 1:
            raise ValueError("the joint model has one coefficient row")
        A = 1 << n_in
        tin = [sum(1 << i for i in range(n_in) if e[j, 1 + i] > 0) for j in range(F)]
        mask = np.array([sum(1 << c for c in range(A) if (tin[j] & ~c) == 0) for j in range(F)], dtype=np.int32)
        exps = e[:, keep]
    return np.ascontiguousarray(mask), np.ascontiguousarray(exps, dtype=np.int8), A


def _refine_rows_call(V, arm, u, seq_len, c0, mask, qexps, A, lib, dt, lam, tau, substeps, revert, outs, nfev, order,
                      n_rows=None):
    """Argument tuple of insite_refine_rows_f64 (the row-layout refinement: no prepare / finish passes)."""
    nul = ctypes.c_void_p(0)
    P_, co, so, io = outs
    N = V.size(0) if n_rows is None else n_rows
    return (_p(V), V.stride(0), V.size(1), _p(arm), arm.stride(0), _p(u) if lib.n_statics else nul, _p(seq_len), N,
            lib.n_statics, int(c0.size), c0.ctypes.data_as(ctypes.c_void_p), mask.ctypes.data_as(ctypes.c_void_p),
            qexps.ctypes.data_as(ctypes.c_void_p), A, float(dt), float(lam), int(tau), int(substeps),
            int(bool(revert)), _p(P_), P_.stride(0), _p(co), _p(so), _p(io), _p(nfev) if nfev is not None else nul,
            _p(order) if order is not None else nul)


def refine_rows_supported(V, arm, u, seq_len, c0, mask, qexps, A, lib, outs) -> bool:
    """Whether insite_refine_rows_f64 takes this model and layout: the library's own answer, asked with zero rows
    (argument and shape checks only, nothing launched).  INSITE_REFINE_ROWS=0 in the environment says no."""
    if A > 4 or os.environ.get("INSITE_REFINE_ROWS", "1") == "0":
        return False
    args = _refine_rows_call(V, arm, u, seq_len, c0, mask, qexps, A, lib, 1.0, 0.0, 0, 1, False, outs, None, None,
                             n_rows=0)
    st = _lib.load().insite_refine_rows_f64(*args, ctypes.c_void_p(0))
    if st == _lib.INSITE_E_UNSUPPORTED:
        return False
    _lib.check("insite_refine_rows_f64", st)
    return True


def insite_refine(V: torch.Tensor, arm: torch.Tensor, u: torch.Tensor, seq_len: torch.Tensor, coef0: np.ndarray,
                  lib: PolyLibrary, dt: float, lam: float, tau: int, substeps: int = 5,
                  revert_on_zoom_fail: bool = False, binned: bool = True, nfev: torch.Tensor | None = None,
                  rows: bool | None = None):
    """INSITE per-patient refinement (reference sindy.py:433-715).  V [N, T] f64 unscaled observations
    and arm [N, T] int8 per-step arms in the reference's patient-major layout (transposed to the
    kernel's time-major layout here), u [N, U], seq_len [N], coef0 the HOST global model [A, F].
    Per-arm models: A <= 2 runs insite_refine_f64 on bit-packed arms, A <= 4 (cancer_sim / EQ_5)
    insite_refine_arms_f64 on int8 arms; libraries with state exponents up to 4 (the degree-4 ablation)
    run the state-polynomial kernels.  The joint model (``lib.n_inputs`` > 0, coef0 [1, F], arm = the
    per-step treatment bit code, ``SINDY._treatment_code``): insite_refine_general_f64 with the folded
    per-coefficient arm masks.  ``revert_on_zoom_fail``: BFGS status 3 falls back to coef0 as
    sindy.py:628-631 reads; the default (False) keeps the iterate, which reproduces the reference's published
    runs.  ``binned``: lanes take the rows sorted by seq_len (insite_rk45_order_i32 on the
    device), so a wave's objective scans have similar lengths; scheduling only, the outputs are bitwise the
    same.  The rows are gathered in lane order by insite_refine_prepare_f64 and the predictions scattered back
    by insite_refine_finish_f64, so every kernel access stays coalesced (round 2's lane -> row indirection
    inside the kernel scattered them: 10.7 vs 9.5 ms).
    ``nfev``: an int32 [N] device tensor receiving each row's objective/gradient evaluation count (the work
    count behind bench.py's INSITE roofline); it routes every model through insite_refine_general_f64 (the
    same kernels and arithmetic as the per-arm entry points).
    ``rows`` (ABI 9): None / True take insite_refine_rows_f64 -- the windowed kernel on the patient-major rows
    themselves, no prepare / finish passes -- whenever the library reports the model and layout in its shape (two
    arms, <= 3 active coefficients, affine RHS, T <= 64); False forces the prepare / kernel / finish route.  The
    outputs are bitwise the same either way.
    Returns (preds [N, T], coef [N, A, F], status [N], iterations [N])."""
    _dev("V", V, torch.float64, 2)
    _dev("arm", arm, torch.int8, 2)
    N, T = V.shape
    if arm.shape != (N, T):
        raise ValueError("arm must be [N, T]")
    if lib.n_statics:
        _dev("u", u, torch.float64, 2)
        if u.size(0) != N or u.size(1) != lib.n_statics or u.stride(0) != lib.n_statics:
            raise ValueError("u must be a contiguous [N, n_statics] tensor")
    _dev("seq_len", seq_len, torch.int32, 1)
    c0 = np.ascontiguousarray(coef0, dtype=np.float64)
    if c0.ndim != 2 or c0.shape[1] != lib.n_terms:
        raise ValueError("coef0 must be a host [A, F] array")
    mask, qexps, A = refine_terms(lib, c0.shape[0])
    if A > 4:
        raise ValueError("at most 4 treatment arms (joint model: 2 binary treatment inputs)")
    if rows is not False:   # (A <= 2: the windowed kernels; 3-4 arms: the cooperative kernel of the dense models)
        if lib.n_statics and u.size(0) != N:
            raise ValueError("u must have one row per refined row")
        if seq_len.numel() != N:
            raise ValueError("seq_len must have one entry per row")
        if nfev is not None:
            _dev("nfev", nfev, torch.int32, 1)
            if nfev.numel() != N:
                raise ValueError("nfev must have one entry per row")
        outs = (torch.empty((N, T), dtype=torch.float64, device=V.device),
                torch.empty((N,) + c0.shape, dtype=torch.float64, device=V.device),
                torch.empty((N,), dtype=torch.int32, device=V.device), torch.empty((N,), dtype=torch.int32, device=V.device))
        if N and V.stride(1) == 1 and arm.stride(1) == 1 and \
                refine_rows_supported(V, arm, u, seq_len, c0, mask, qexps, A, lib, outs):
            if A <= 2 and int(arm.amax().item()) > 1:
                raise ValueError("two-arm models need arm values 0/1")
            order = rk45_order(seq_len, T) if (binned and N > 64) else None
            args = _refine_rows_call(V, arm, u, seq_len, c0, mask, qexps, A, lib, dt, lam, tau, substeps,
                                     revert_on_zoom_fail, outs, nfev, order)
            _run(("insite_refine_rows_f64", args, V.device, None))
            return outs
        if rows:
            raise ValueError("insite_refine_rows_f64 does not take this model / layout (INSITE_E_UNSUPPORTED)")
    order = rk45_order(seq_len, T) if (binned and N > 64) else None
    if order is None:
        Vt, arms = refine_prepare(V, arm, bits=A <= 2, order=None)
        preds, coef, status, iters = insite_refine_tm(Vt, arms, u, seq_len, c0, lib, dt, lam, tau, substeps,
                                                      revert_on_zoom_fail, nfev=nfev)
        return preds.t(), coef, status, iters
    # binned: the rows (with their statics and sequence lengths) are gathered in lane order by ONE prepare pass,
    # the kernel runs the identity order on them (coalesced loads and stores), and ONE finish pass scatters the
    # predictions, coefficients, statuses and iteration counts back to row order
    Vt, arms, u_l, sl_l = refine_prepare(V, arm, bits=A <= 2, order=order, u=u if lib.n_statics else None,
                                         seq_len=seq_len)
    nf = torch.empty_like(nfev) if nfev is not None else None
    preds, coef, status, iters = insite_refine_tm(Vt, arms, u_l if lib.n_statics else u, sl_l, c0, lib, dt, lam, tau,
                                                  substeps, revert_on_zoom_fail, nfev=nf)
    if nfev is not None:
        nfev.index_copy_(0, order.long(), nf)
    return refine_finish(preds, order, N, lane_outputs=(coef, status, iters))


class InsiteRefinePlan:
    """``insite_refine`` (binned) prepared once: the inputs validated (the arm range check included) and every buffer
    and argument packed, so a call enqueues two C calls in the row layout (``mode`` "rows", ABI 9: the seq_len
    counting sort and insite_refine_rows_f64) or else four -- the seq_len counting sort
    (insite_rk45_order_i32), the gather pass (insite_refine_prepare_f64: rows, statics, sequence lengths into lane
    order), the refinement kernel, and the scatter pass (insite_refine_finish_f64: predictions, coefficients,
    statuses, iteration counts back to row order) -- with no host synchronisation.  Outputs ``out`` = (preds
    [N, T], coef [N, A, F], status [N], iters [N]), bitwise those of ``insite_refine``.  The plan keeps references
    to its inputs: refresh them in place between calls (a serving loop) or make a new plan."""

    def __init__(self, V, arm, u, seq_len, coef0, lib, dt, lam, tau, substeps=5, revert_on_zoom_fail=False,
                 rows=None, nfev=None, order="seq_len"):
        L = _lib.load()
        if order not in ("seq_len", "nfev"):
            raise ValueError("order must be 'seq_len' or 'nfev'")
        _dev("V", V, torch.float64, 2)
        _dev("arm", arm, torch.int8, 2)
        N, T = V.shape
        if arm.shape != (N, T) or V.stride(1) != 1 or arm.stride(1) != 1 or N < 1:
            raise ValueError("V and arm must be row-contiguous [N >= 1, T]")
        _dev("seq_len", seq_len, torch.int32, 1)
        if seq_len.numel() != N:
            raise ValueError("seq_len must have one entry per row")
        if lib.n_statics:
            _dev("u", u, torch.float64, 2)
            if u.size(0) != N or u.size(1) != lib.n_statics or not u.is_contiguous():
                raise ValueError("u must be a contiguous [N, n_statics] tensor")
        c0 = np.ascontiguousarray(coef0, dtype=np.float64)
        if c0.ndim != 2 or c0.shape[1] != lib.n_terms:
            raise ValueError("coef0 must be a host [A, F] array")
        mask, qexps, A = refine_terms(lib, c0.shape[0])
        if A > 4:
            raise ValueError("at most 4 treatment arms (joint model: 2 binary treatment inputs)")
        bits = A <= 2
        if bits and int(arm.amax().item()) > 1:          # once, here: the calls never synchronise
            raise ValueError("bit-packed arms need n_arms <= 2 (arm values 0/1)")
        dev = V.device
        W = (N + 31) // 32
        U = lib.n_statics
        self.order = torch.empty((N,), dtype=torch.int32, device=dev)
        self._ows = Workspace("scratch").get(L.insite_rk45_order_workspace_bytes(int(T)), dev)
        self._c0, self._mask, self._qexps, self._tab = c0, mask, qexps, lib.ctypes_table()
        self.device = dev
        order_call = (L.insite_rk45_order_i32, (_p(seq_len), N, int(T), _p(self.order), _p(self._ows),
                                                self._ows.numel()))
        if nfev is not None:
            _dev("nfev", nfev, torch.int32, 1)
            if nfev.numel() != N:
                raise ValueError("nfev must have one entry per row")
        key_call = None
        self.nfev = None   # (order="nfev": the evaluation counts the binning key reads, rewritten by every call)
        if order == "nfev":
            # lanes binned by the window (seq_len, 32 levels) and then by the evaluation counts the previous call left
            # in ``nfev`` (32 levels): a wave runs until its longest row's last objective scan, so rows of equal window
            # AND equal evaluation count belong together (the C5 line's attempt binning; a refined set that is refined
            # again -- the bench step, a serving loop -- takes the same counts).  Outputs do not depend on the lane
            # order (tested); the first call bins on zero counts, i.e. by seq_len alone.
            if nfev is None:
                nfev = torch.zeros((N,), dtype=torch.int32, device=dev)
            self._key = torch.empty((N,), dtype=torch.int32, device=dev)
            key, sl_, nf_, Tq = self._key, seq_len, nfev, max(int(T), 1)
            kws = Workspace("scratch").get(L.insite_rk45_order_workspace_bytes(RK45_ATTEMPT_BINS - 1), dev)
            self._kws = kws

            # key resolution: window levels x evaluation-count levels = 1,024 bins (INSITE_NFEV_KEY "32x32", the
            # default: the window in 32 levels, min(nfev, 31) -- wave divergence 1.025 at the INSITE line's shape;
            # "64x16": the window in 64 levels, min(nfev / 2, 15) -- 1.056, 1.5-2.7 % slower, profiles/r06/nfkey/)
            wl, nl = (64, 16) if os.environ.get("INSITE_NFEV_KEY", "32x32") == "64x16" else (32, 32)
            nsh = 0 if nl == 32 else 1

            def key_fn(s):   # key = window level * nl + min(nfev >> nsh, nl - 1) in [0, 1024), on the plan's stream s
                with torch.cuda.stream(s):
                    q = torch.clamp(sl_, 0, Tq).mul_(wl - 1).floor_divide_(Tq).mul_(nl)
                    torch.add(q, torch.clamp(nf_ >> nsh, 0, nl - 1), out=key)
            key_call = (key_fn, None)
            self.nfev = nfev
            order_call = (L.insite_rk45_order_i32, (_p(key), N, RK45_ATTEMPT_BINS - 1, _p(self.order), _p(kws),
                                                    kws.numel()))
        self._keep = (V, arm, u, seq_len, nfev)
        if rows is not False:   # (3-4 arms: the cooperative kernel's row layout where the library takes the model)
            outs = (torch.empty((N, T), dtype=torch.float64, device=dev),
                    torch.empty((N,) + c0.shape, dtype=torch.float64, device=dev),
                    torch.empty((N,), dtype=torch.int32, device=dev), torch.empty((N,), dtype=torch.int32, device=dev))
            if refine_rows_supported(V, arm, u, seq_len, c0, mask, qexps, A, lib, outs):
                # the row layout (ABI 9): two C calls, the counting sort and the refinement on the rows themselves
                self.mode = "rows"
                self.out = outs
                self.kernel_call = 2 if key_call else 1   # (the refinement kernel's index in _calls)
                self._calls = ([key_call] if key_call else []) + [order_call, (L.insite_refine_rows_f64, _refine_rows_call(
                    V, arm, u, seq_len, c0, mask, qexps, A, lib, dt, lam, tau, substeps, revert_on_zoom_fail, outs,
                    nfev, self.order))]
                return
            if rows:
                raise ValueError("insite_refine_rows_f64 does not take this model / layout (INSITE_E_UNSUPPORTED)")
        if nfev is not None and key_call is None:
            raise ValueError("nfev needs the row-layout plan (or order='nfev')")
        self.mode = "prepare"
        self.kernel_call = 3 if key_call else 2
        # order="nfev": the kernel counts evaluations per lane (the general entry point, the same kernels), a last
        # torch step scatters them to row order for the next call's key
        self.nf_lane = torch.zeros((N,), dtype=torch.int32, device=dev) if key_call else None
        ldt = N + (N & 1)   # even leading dimension (the windowed kernels' 16-B ring loads)
        self.Vt = torch.empty((T, ldt), dtype=torch.float64, device=dev)[:, :N]
        self.arms = torch.empty((T, W) if bits else (T, N), dtype=torch.int32 if bits else torch.int8, device=dev)
        self.u_l = torch.empty_like(u) if U else None
        self.sl_l = torch.empty_like(seq_len)
        self.P = torch.empty((T, N), dtype=torch.float64, device=dev)
        self.coef_l = torch.empty((N,) + c0.shape, dtype=torch.float64, device=dev)
        self.st_l = torch.empty((N,), dtype=torch.int32, device=dev)
        self.it_l = torch.empty((N,), dtype=torch.int32, device=dev)
        self.out = (torch.empty((N, T), dtype=torch.float64, device=dev), torch.empty_like(self.coef_l),
                    torch.empty_like(self.st_l), torch.empty_like(self.it_l))
        nul = ctypes.c_void_p(0)
        self._calls = ([key_call] if key_call else []) + [
            order_call,
            (L.insite_refine_prepare_f64, (_p(V), V.stride(0), _p(arm), arm.stride(0), N, T, _p(self.Vt), ldt,
                                           _p(self.arms) if bits else nul, W, nul if bits else _p(self.arms), N,
                                           _p(self.order), _p(u) if U else nul, U, _p(self.u_l) if U else nul,
                                           _p(seq_len), _p(self.sl_l))),
        ]
        common = (float(dt), float(lam), int(tau), int(substeps), int(bool(revert_on_zoom_fail)), _p(self.P), N,
                  _p(self.coef_l), _p(self.st_l), _p(self.it_l))
        ustat = _p(self.u_l) if U else nul
        if lib.n_inputs or key_call:
            self._calls.append((L.insite_refine_general_f64, (
                _p(self.Vt), ldt, T, _p(self.arms) if bits else nul, nul if bits else _p(self.arms), self.arms.stride(0),
                ustat, _p(self.sl_l), N, U, c0.size, c0.ctypes.data_as(ctypes.c_void_p),
                mask.ctypes.data_as(ctypes.c_void_p), qexps.ctypes.data_as(ctypes.c_void_p), A) + common +
                (_p(self.nf_lane) if key_call else nul, nul)))
        else:
            fn = L.insite_refine_f64 if bits else L.insite_refine_arms_f64
            self._calls.append((fn, (_p(self.Vt), ldt, T, _p(self.arms), self.arms.stride(0), ustat, _p(self.sl_l), N, U,
                                     self._tab.ctypes.data_as(ctypes.c_void_p), lib.n_terms,
                                     c0.ctypes.data_as(ctypes.c_void_p), A) + common + (nul,)))
        P_, co, so, io = self.out
        self._calls.append((L.insite_refine_finish_f64, (_p(self.P), N, _p(self.order), N, T, _p(P_), T,
                                                         _p(self.coef_l), int(c0.size), _p(co), _p(self.st_l), _p(so),
                                                         _p(self.it_l), _p(io))))
        if key_call:
            nf_row, nf_l, ordr = self.nfev, self.nf_lane, self.order

            def nfev_scatter(s):   # lane counts -> row order (the next call's key)
                with torch.cuda.stream(s):
                    nf_row.index_copy_(0, ordr.long(), nf_l)
            self._calls.append((nfev_scatter, None))

    def __call__(self, stream: torch.cuda.Stream | None = None):
        for i in range(len(self._calls)):
            self.call(i, stream)
        return self.out

    def call(self, i: int, stream: torch.cuda.Stream | None = None):
        """Enqueue the plan's i-th C call alone (bench.py times the refinement kernel this way)."""
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        fn, args = self._calls[i]
        if args is None:   # a torch step (the nfev binning key): its ops on the same stream
            fn(s)
            return
        st = fn(*args, ctypes.c_void_p(s.cuda_stream))
        if st:
            _lib.check(getattr(fn, "__name__", "insite refine plan"), st)


def plan_insite_refine(V, arm, u, seq_len, coef0, lib, dt, lam, tau, substeps=5, revert_on_zoom_fail=False,
                       rows=None, nfev=None, order="seq_len"):
    """``insite_refine`` (binned lane order) as a prepared plan (``InsiteRefinePlan``).  ``rows`` as in
    ``insite_refine``; ``nfev`` (row layout only) an int32 [N] tensor receiving each row's evaluation count;
    ``order`` "seq_len" (lanes binned by the row's window) or "nfev" (by the window, then by the evaluation counts
    the previous call left in ``nfev``)."""
    return InsiteRefinePlan(V, arm, u, seq_len, coef0, lib, dt, lam, tau, substeps, revert_on_zoom_fail, rows, nfev,
                            order)


def refine_prepare(V: torch.Tensor, arm: torch.Tensor, bits: bool = True, order: torch.Tensor | None = None,
                   u: torch.Tensor | None = None, seq_len: torch.Tensor | None = None, check: bool = True):
    """Patient-major V [N, T] f64 and per-step arms [N, T] int8 -> the refinement kernels' time-major Vt [T, N] and
    arms (bit-packed int32 [T, ceil(N / 32)] when ``bits``, else int8 [T, N]) in one device pass
    (insite_refine_prepare_f64).  Bit-packing needs arm values 0 / 1 (checked here: two arms, or the joint
    model's combination codes of one binary input; ``check=False`` skips that device-to-host check for a caller
    that validated the arms once).  ``order`` [N] int32: output column l takes row order[l]; with ``u`` [N, U]
    and / or ``seq_len`` [N] the same pass gathers them too and the result is (Vt, arms, u_l, seq_len_l)."""
    _dev("V", V, torch.float64, 2)
    _dev("arm", arm, torch.int8, 2)
    N, T = V.shape
    if arm.shape != (N, T) or V.stride(1) != 1 or arm.stride(1) != 1:
        raise ValueError("V and arm must be row-contiguous [N, T]")
    if check and bits and N and int(arm.amax().item()) > 1:
        raise ValueError("bit-packed arms need n_arms <= 2 (arm values 0/1)")
    side = u is not None or seq_len is not None
    u_l = sl_l = None
    if u is not None:
        _dev("u", u, torch.float64, 2)
        if u.size(0) != N or not u.is_contiguous():
            raise ValueError("u must be a contiguous [N, n_statics] tensor")
        u_l = torch.empty_like(u)
    if seq_len is not None:
        _dev("seq_len", seq_len, torch.int32, 1)
        if seq_len.numel() != N:
            raise ValueError("seq_len must have one entry per row")
        sl_l = torch.empty_like(seq_len)
    ldt = N + (N & 1)   # an even leading dimension: the windowed kernels' 16-B ring loads (insite_refine.hip)
    Vt = torch.empty((T, ldt), dtype=torch.float64, device=V.device)[:, :N]
    W = (N + 31) // 32
    at = torch.empty((T, W) if bits else (T, N), dtype=torch.int32 if bits else torch.int8, device=V.device)
    nul = ctypes.c_void_p(0)
    if order is not None:
        _dev("order", order, torch.int32, 1)
        if order.numel() != N:
            raise ValueError("order must be an [N] permutation")
    st = _lib.load().insite_refine_prepare_f64(_p(V), V.stride(0), _p(arm), arm.stride(0), N, T, _p(Vt), ldt,
                                               _p(at) if bits else nul, W, nul if bits else _p(at), N, _p(order),
                                               _p(u), u.size(1) if u is not None else 0, _p(u_l), _p(seq_len), _p(sl_l),
                                               _stream(V.device))
    _lib.check("insite_refine_prepare_f64", st)
    return (Vt, at, u_l, sl_l) if side else (Vt, at)


def refine_finish(P: torch.Tensor, order: torch.Tensor | None, N: int, lane_outputs: tuple | None = None):
    """Time-major refinement predictions P [T, >= N] whose column l is row order[l] (identity when None) ->
    patient-major [N, T] (insite_refine_finish_f64).  ``lane_outputs`` = (coef [N, ...] f64, status [N] int32,
    iters [N] int32) in lane order: the same pass scatters them back to row order and the result is
    (preds, coef, status, iters)."""
    _dev("P", P, torch.float64, 2)
    T = P.size(0)
    if P.size(1) < N or P.stride(1) != 1:
        raise ValueError("P must be row-contiguous [T, >= N]")
    if order is not None:
        _dev("order", order, torch.int32, 1)
    out = torch.empty((N, T), dtype=torch.float64, device=P.device)
    nul = ctypes.c_void_p(0)
    if lane_outputs is not None:
        c, s_, it = lane_outputs
        _dev("coef", c, torch.float64)
        _dev("status", s_, torch.int32, 1)
        _dev("iters", it, torch.int32, 1)
        if c.size(0) != N or not c.is_contiguous() or s_.numel() != N or it.numel() != N:
            raise ValueError("lane outputs must have one contiguous row per refined row")
        co, so, io = torch.empty_like(c), torch.empty_like(s_), torch.empty_like(it)
        nc = c.numel() // max(N, 1)
        extra = (_p(c), nc, _p(co), _p(s_), _p(so), _p(it), _p(io))
    else:
        extra = (nul, 0, nul, nul, nul, nul, nul)
    st = _lib.load().insite_refine_finish_f64(_p(P), P.stride(0), _p(order), N, T, _p(out), T, *extra,
                                              _stream(P.device))
    _lib.check("insite_refine_finish_f64", st)
    return (out, co, so, io) if lane_outputs is not None else out


def insite_refine_tm(Vt: torch.Tensor, arms: torch.Tensor, u: torch.Tensor, seq_len: torch.Tensor, coef0,
                     lib: PolyLibrary, dt: float, lam: float, tau: int, substeps: int = 5,
                     revert_on_zoom_fail: bool = False, order: torch.Tensor | None = None,
                     nfev: torch.Tensor | None = None):
    """``insite_refine`` on the kernels' own time-major layout (no per-call transposes): Vt [T, >= N] f64, arms
    the per-step arms as the bit mask int32 [T, >= ceil(N / 32)] (A <= 2, ``pack_arm_bits``) or int8 [T, >= N]
    (A <= 4); ``order`` an optional lane -> row permutation (``rk45_order``).  Returns (preds [T, N] time-major,
    coef [N, A, F], status [N], iterations [N])."""
    _dev("Vt", Vt, torch.float64, 2)
    _dev("seq_len", seq_len, torch.int32, 1)
    N = seq_len.numel()
    T = Vt.size(0)
    if Vt.size(1) < N:
        raise ValueError("Vt must be [T, >= N]")
    c0 = np.ascontiguousarray(coef0, dtype=np.float64)
    if c0.ndim != 2 or c0.shape[1] != lib.n_terms:
        raise ValueError("coef0 must be a host [A, F] array")
    mask, qexps, A = refine_terms(lib, c0.shape[0])
    if A > 4:
        raise ValueError("at most 4 treatment arms (joint model: 2 binary treatment inputs)")
    if A <= 2:
        _dev("arms", arms, torch.int32, 2)
        if arms.size(0) < T or arms.size(1) < (N + 31) // 32:
            raise ValueError("bit-packed arms must be [T, >= ceil(N / 32)] int32")
    else:
        _dev("arms", arms, torch.int8, 2)
        if arms.size(0) < T or arms.size(1) < N:
            raise ValueError("int8 arms must be [T, >= N]")
    if lib.n_statics:
        _dev("u", u, torch.float64, 2)
        if u.size(0) != N or u.size(1) != lib.n_statics or u.stride(0) != lib.n_statics:
            raise ValueError("u must be a contiguous [N, n_statics] tensor")
    if nfev is not None:
        _dev("nfev", nfev, torch.int32, 1)
        if nfev.numel() != N:
            raise ValueError("nfev must have one entry per row")
    dev = Vt.device
    preds = torch.empty((T, N), dtype=torch.float64, device=dev)
    coef = torch.empty((N,) + c0.shape, dtype=torch.float64, device=dev)
    status = torch.empty((N,), dtype=torch.int32, device=dev)
    iters = torch.empty((N,), dtype=torch.int32, device=dev)
    nul = ctypes.c_void_p(0)
    ustat = _p(u) if lib.n_statics else nul
    tail = (c0.ctypes.data_as(ctypes.c_void_p),)
    common = (float(dt), float(lam), int(tau), int(substeps), int(bool(revert_on_zoom_fail)), _p(preds),
              preds.stride(0), _p(coef), _p(status), _p(iters), _p(order) if order is not None else nul)
    if lib.n_inputs or nfev is not None:
        gcommon = common[:-1] + (_p(nfev), common[-1])
        args = (_p(Vt), Vt.stride(0), T, _p(arms) if A <= 2 else nul, _p(arms) if A > 2 else nul, arms.stride(0),
                ustat, _p(seq_len), N, lib.n_statics, c0.size, *tail, mask.ctypes.data_as(ctypes.c_void_p),
                qexps.ctypes.data_as(ctypes.c_void_p), A) + gcommon
        _run(("insite_refine_general_f64", args, dev, None))
    else:
        tab = lib.ctypes_table()
        name = "insite_refine_f64" if A <= 2 else "insite_refine_arms_f64"
        args = (_p(Vt), Vt.stride(0), T, _p(arms), arms.stride(0), ustat, _p(seq_len), N, lib.n_statics,
                tab.ctypes.data_as(ctypes.c_void_p), lib.n_terms, *tail, A) + common
        _run((name, args, dev, None))
    return preds, coef, status, iters


def masked_sse(pred: torch.Tensor, target: torch.Tensor, active: torch.Tensor, scale: float = 1.0,
               shift: float = 0.0, workspace: Workspace | None = None):
    """Masked squared-error sums (insite_masked_sse_f64).  Returns (per_step[T], count[T], last[2])."""
    L = _lib.load()
    _dev("pred", pred, torch.float64, 2)
    _dev("target", target, torch.float64, 2)
    _dev("active", active, torch.float64, 2)
    N, T = target.shape
    if not target.is_contiguous() or not active.is_contiguous() or active.shape != target.shape:
        raise ValueError("target/active must be contiguous [N,T]")
    if pred.size(0) != N or pred.size(1) < T:
        raise ValueError("pred must be [N, >=T]")
    per = torch.empty(T, dtype=torch.float64, device=pred.device)
    cnt = torch.empty(T, dtype=torch.float64, device=pred.device)
    last = torch.empty(2, dtype=torch.float64, device=pred.device)
    nbytes = L.insite_masked_sse_workspace_bytes(N, T)
    ws = _ws(workspace, pred.device, "scratch").get(nbytes, pred.device)
    st = L.insite_masked_sse_f64(_p(pred), pred.stride(0), float(scale), float(shift), _p(target), _p(active), N, T,
                                 _p(per), _p(cnt), _p(last), _p(ws), ws.numel(), _stream(pred.device))
    _lib.check("insite_masked_sse_f64", st)
    return per, cnt, last


def poly_library_native(n_statics: int, degree: int, interaction_only: bool) -> np.ndarray:
    """The library exponent table as produced by the C ABI (host function, no GPU needed)."""
    L = _lib.load()
    n_in = 1 + n_statics
    buf = np.zeros((256, n_in), dtype=np.int8)
    n = ctypes.c_int32(0)
    st = L.insite_poly_library(n_statics, degree, int(interaction_only), buf.ctypes.data_as(ctypes.c_void_p), 256,
                               ctypes.byref(n))
    _lib.check("insite_poly_library", st)
    return buf[: n.value].copy()
