"""ctypes binding of ``libinsite_hip.so`` (the C ABI declared in ``include/insite_hip.h``).

The product path has no CPU fallback: if the shared library is missing or cannot be loaded
every op raises ``InsiteLibraryError``.  ``torch`` is imported first so that the library binds
to the HIP runtime torch already loaded (same soname ``libamdhip64.so.7``) and torch stream
handles are valid across the ABI.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the dlopen below: shared HIP runtime)

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(PKG_ROOT, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libinsite_hip.so")
# profiling-only override (ablation builds under tools/); never set in product runs
if os.environ.get("INSITE_LIB_OVERRIDE"):
    LIB_PATH = os.environ["INSITE_LIB_OVERRIDE"]

ABI_VERSION = 9

# status codes / enums (insite_hip.h)
INSITE_OK = 0
INSITE_E_UNSUPPORTED = -2   # include/insite_hip.h
FD_SMOOTHED4, FD_ORDER4, FD_ORDER1, FD_SMOOTHED1 = 0, 1, 2, 3
METHOD_EULER, METHOD_RK4 = 0, 1
LAYOUT_PATIENT_MAJOR, LAYOUT_TIME_MAJOR, LAYOUT_TIME_MAJOR_BITS, LAYOUT_PATIENT_MAJOR_BITS = 0, 1, 2, 3
MAX_TERMS, MAX_STATICS, MAX_ARMS, MAX_STATE_DEGREE = 9, 3, 4, 1
GEN_MAX_TERMS, GEN_MAX_STATE_DEGREE, GEN_MAX_INPUTS = 64, 4, 2   # insite_gen.hip

EXPORTS = (
    "insite_abi_version",
    "insite_strerror",
    "insite_poly_library",
    "insite_gram_workspace_bytes",
    "insite_gram_f64",
    "insite_sindy_fit_f64",
    "insite_fit_rollout_f64",
    "insite_fit_rollout_deferred_workspace_bytes",
    "insite_fit_rollout_deferred_f64",
    "insite_fit_rollout_lagged_f64",
    "insite_gram_segments_workspace_bytes",
    "insite_gram_segments_f64",
    "insite_sindy_fit_segments_f64",
    "insite_per_patient_workspace_bytes",
    "insite_sindy_fit_per_patient_f64",
    "insite_gram_moments_f64",
    "insite_fit_per_patient_moments_f64",
    "insite_stlsq_f64",
    "insite_rollout_f64",
    "insite_rollout_rk45_f64",
    "insite_rk45_order_workspace_bytes",
    "insite_rk45_order_i32",
    "insite_refine_f64",
    "insite_refine_arms_f64",
    "insite_refine_general_f64",
    "insite_refine_rows_f64",
    "insite_refine_prepare_f64",
    "insite_refine_finish_f64",
    "insite_gen_gram_segments_workspace_bytes",
    "insite_gen_gram_segments_f64",
    "insite_masked_sse_workspace_bytes",
    "insite_masked_sse_f64",
    "insite_gram_ms_workspace_bytes",
    "insite_gram_ms_f32",
    "insite_stlsq_wave_f64",
    "insite_rollout_ms_f32",
    "insite_rollout_ms_sparse_f32",
    "insite_gen_gram_workspace_bytes",
    "insite_gen_gram_f64",
    "insite_stlsq_wave64_f64",
    "insite_rollout_poly_f64",
    "insite_threefry2x32_iota_u32",
    "insite_refit_rollout_moments_f64",
)


class InsiteLibraryError(RuntimeError):
    pass


class InsiteError(RuntimeError):
    def __init__(self, fn, code, msg):
        super().__init__(f"{fn} failed with status {code}: {msg}")
        self.code = code


_lock = threading.Lock()
_lib = None

_c_i32, _c_i64, _c_f64, _c_size, _vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_size_t, ctypes.c_void_p

_SIGNATURES = {
    "insite_abi_version": (_c_i32, []),
    "insite_strerror": (ctypes.c_char_p, [_c_i32]),
    "insite_poly_library": (_c_i32, [_c_i32, _c_i32, _c_i32, _vp, _c_i32, ctypes.POINTER(_c_i32)]),
    "insite_gram_workspace_bytes": (_c_size, [_c_i64, _c_i32, _c_i32]),
    "insite_gram_f64": (_c_i32, [_vp, _c_i64, _c_i32, _c_i32, _vp, _vp, _vp, _c_i64, _c_i32, _c_i32, _vp, _c_i32,
                                 _c_i32, _c_f64, _vp, _vp, _vp, _c_size, _vp]),
    "insite_sindy_fit_f64": (_c_i32, [_vp, _c_i64, _c_i32, _c_i32, _vp, _vp, _vp, _c_i64, _c_i32, _c_i32, _vp,
                                      _c_i32, _c_i32,
                                      _c_f64, _c_f64, _c_f64, _c_i32, _c_i32, _vp, _vp, _vp, _vp, _vp, _vp, _c_size,
                                      _vp]),
    "insite_fit_rollout_f64": (_c_i32, [_vp, _c_i64, _c_i32, _vp, _vp, _vp, _c_i64, _c_i32, _c_i32, _vp, _c_i32,
                                        _c_i32, _c_f64, _c_f64, _c_f64, _c_i32, _c_i32, _vp, _vp, _vp, _vp, _vp,
                                        _vp, _vp, _vp, _c_i64, _vp, _c_i64, _c_i32, _c_f64, _c_i32, _c_i32, _c_f64,
                                        _vp, _c_i64, _c_i32, _vp, _c_size, _vp]),
    "insite_fit_rollout_deferred_workspace_bytes": (_c_size, [_c_i64, _c_i32, _c_i32]),
    "insite_fit_rollout_deferred_f64": (_c_i32, [_vp, _c_i64, _c_i32, _vp, _vp, _vp, _c_i64, _c_i32, _c_i32, _vp,
                                                 _c_i32, _c_i32, _c_f64, _c_f64, _c_f64, _c_i32, _c_i32, _vp, _vp, _vp,
                                                 _vp, _vp, _vp, _vp, _vp, _c_i64, _vp, _c_i64, _c_i32, _c_f64, _c_i32,
                                                 _c_i32, _c_f64, _vp, _c_i64, _c_i32, _c_i32, _c_i32, _vp, _c_size,
                                                 _vp]),
    "insite_fit_rollout_lagged_f64": (_c_i32, [_vp, _c_i64, _c_i32, _vp, _vp, _vp, _c_i64, _c_i32, _c_i32, _vp,
                                               _c_i32, _c_i32, _c_f64, _c_f64, _c_f64, _c_i32, _c_i32, _vp, _vp, _vp,
                                               _vp, _vp, _vp, _vp, _vp, _vp, _vp, _c_i64, _vp, _c_i64, _c_i32, _c_f64,
                                               _c_i32, _c_i32, _c_f64, _vp, _c_i64, _c_i32, _c_i32, _c_i32, _vp,
                                               _c_size, _vp]),
    "insite_gram_segments_workspace_bytes": (_c_size, [_c_i64, _c_i32, _c_i32]),
    "insite_gram_segments_f64": (_c_i32, [_vp, _c_i64, _vp, _c_i64, _c_i32, _c_i32, _vp, _vp, _c_i64, _c_i32, _c_i32,
                                          _vp, _c_i32, _c_i32, _c_f64, _vp, _vp, _vp, _c_size, _vp]),
    "insite_sindy_fit_segments_f64": (_c_i32, [_vp, _c_i64, _vp, _c_i64, _c_i32, _c_i32, _vp, _vp, _c_i64, _c_i32,
                                               _c_i32, _vp, _c_i32, _c_i32, _c_f64, _c_f64, _c_f64, _c_i32, _c_i32,
                                               _vp, _vp, _vp, _vp, _vp, _vp, _c_size, _vp]),
    "insite_per_patient_workspace_bytes": (_c_size, [_c_i64]),
    "insite_sindy_fit_per_patient_f64": (_c_i32, [_vp, _c_i64, _c_i32, _c_i32, _vp, _vp, _vp, _c_i64, _c_i32, _c_i32,
                                                  _vp, _c_i32, _c_i32, _c_f64, _vp, _c_f64, _c_f64, _c_i32, _c_i32,
                                                  _vp, _vp, _vp, _vp, _c_size, _vp]),
    "insite_gram_moments_f64": (_c_i32, [_vp, _c_i64, _c_i32, _c_i32, _vp, _vp, _vp, _c_i64, _c_i32, _c_i32, _vp,
                                         _c_i32, _c_i32, _c_f64, _c_f64, _c_f64, _c_i32, _c_i32, _vp, _vp, _vp, _vp,
                                         _vp, _vp, _vp, _c_size, _vp]),
    "insite_fit_per_patient_moments_f64": (_c_i32, [_vp, _vp, _vp, _vp, _c_i64, _c_i32, _c_i32, _c_i32, _vp, _c_i32,
                                                    _vp, _c_f64, _c_f64, _c_i32, _c_i32, _vp, _vp, _vp, _vp]),
    "insite_stlsq_f64": (_c_i32, [_vp, _vp, _c_i64, _c_i32, _c_f64, _c_f64, _c_i32, _c_i32, _vp, _vp, _vp, _vp]),
    "insite_rollout_f64": (_c_i32, [_vp, _vp, _vp, _c_i64, _vp, _c_i64, _vp, _c_i32, _c_i64, _c_i32, _c_i32,
                                    _c_i32, _c_f64, _c_i32, _c_i32, _c_f64, _vp, _c_i64, _c_i32, _vp]),
    "insite_rollout_rk45_f64": (_c_i32, [_vp, _vp, _vp, _c_i64, _vp, _c_i64, _vp, _vp, _c_i64, _vp, _c_i32, _c_i64,
                                         _c_i32, _c_i32, _c_i32, _c_f64, _c_f64, _c_f64, _vp, _c_i64, _vp, _vp,
                                         _c_i32, _vp]),
    "insite_rk45_order_workspace_bytes": (_c_size, [_c_i32]),
    "insite_rk45_order_i32": (_c_i32, [_vp, _c_i64, _c_i32, _vp, _vp, _c_size, _vp]),
    "insite_refine_f64": (_c_i32, [_vp, _c_i64, _c_i32, _vp, _c_i64, _vp, _vp, _c_i64, _c_i32, _vp, _c_i32, _vp,
                                   _c_i32, _c_f64, _c_f64, _c_i32, _c_i32, _c_i32, _vp, _c_i64, _vp, _vp, _vp, _vp,
                                   _vp]),
    "insite_refine_arms_f64": (_c_i32, [_vp, _c_i64, _c_i32, _vp, _c_i64, _vp, _vp, _c_i64, _c_i32, _vp, _c_i32,
                                        _vp, _c_i32, _c_f64, _c_f64, _c_i32, _c_i32, _c_i32, _vp, _c_i64, _vp, _vp, _vp,
                                        _vp, _vp]),
    "insite_refine_general_f64": (_c_i32, [_vp, _c_i64, _c_i32, _vp, _vp, _c_i64, _vp, _vp, _c_i64, _c_i32, _c_i32,
                                           _vp, _vp, _vp, _c_i32, _c_f64, _c_f64, _c_i32, _c_i32, _c_i32, _vp, _c_i64,
                                           _vp, _vp, _vp, _vp, _vp, _vp]),
    "insite_refine_rows_f64": (_c_i32, [_vp, _c_i64, _c_i32, _vp, _c_i64, _vp, _vp, _c_i64, _c_i32, _c_i32, _vp,
                                        _vp, _vp, _c_i32, _c_f64, _c_f64, _c_i32, _c_i32, _c_i32, _vp, _c_i64, _vp,
                                        _vp, _vp, _vp, _vp, _vp]),
    "insite_refine_prepare_f64": (_c_i32, [_vp, _c_i64, _vp, _c_i64, _c_i64, _c_i32, _vp, _c_i64, _vp, _c_i64, _vp,
                                           _c_i64, _vp, _vp, _c_i32, _vp, _vp, _vp, _vp]),
    "insite_refine_finish_f64": (_c_i32, [_vp, _c_i64, _vp, _c_i64, _c_i32, _vp, _c_i64, _vp, _c_i32, _vp, _vp, _vp,
                                          _vp, _vp, _vp]),
    "insite_gen_gram_segments_workspace_bytes": (_c_size, [_c_i64, _c_i32, _c_i32]),
    "insite_gen_gram_segments_f64": (_c_i32, [_vp, _c_i64, _vp, _c_i64, _c_i32, _c_i32, _vp, _vp, _c_i32, _c_i64,
                                              _c_i32, _vp, _c_i32, _c_i32, _c_f64, _vp, _vp, _vp, _c_size, _vp]),
    "insite_refit_rollout_moments_f64": (_c_i32, [_vp, _vp, _vp, _c_i64, _c_i32, _c_i32, _c_i32, _vp, _c_i32, _vp,
                                                  _c_f64, _c_f64, _c_i32, _c_i32, _vp, _vp, _vp, _c_i64, _c_i32,
                                                  _c_f64, _c_i32, _c_i32, _c_f64, _vp, _c_i64, _vp, _vp, _vp, _vp]),
    "insite_threefry2x32_iota_u32": (_c_i32, [ctypes.c_uint32, ctypes.c_uint32, _c_i64, _vp, _vp]),
    "insite_masked_sse_workspace_bytes": (_c_size, [_c_i64, _c_i32]),
    "insite_masked_sse_f64": (_c_i32, [_vp, _c_i64, _c_f64, _c_f64, _vp, _vp, _c_i64, _c_i32, _vp, _vp, _vp,
                                       _vp, _c_size, _vp]),
    "insite_gram_ms_workspace_bytes": (_c_size, [_c_i64]),
    "insite_gram_ms_f32": (_c_i32, [_vp, _c_i64, _c_i32, _c_i32, _vp, _c_i64, _vp, _c_i64, _vp, _c_i32, _c_i32,
                                    _c_f64, _vp, _vp, _vp, _c_size, _vp]),
    "insite_stlsq_wave_f64": (_c_i32, [_vp, _vp, _c_i32, _c_i32, _c_f64, _c_f64, _c_i32, _c_i32, _vp, _vp, _vp,
                                       _vp]),
    "insite_rollout_ms_f32": (_c_i32, [_vp, _c_i64, _vp, _c_i64, _vp, _vp, _c_i32, _c_i32, _c_i64, _c_i32, _c_f64,
                                       _c_i32, _c_i32, _c_f64, _vp, _c_i64, _vp]),
    "insite_rollout_ms_sparse_f32": (_c_i32, [_vp, _c_i64, _vp, _c_i64, _vp, _vp, _vp, _c_i32, _c_i32, _c_i64, _c_i32,
                                              _c_f64, _c_i32, _c_i32, _c_f64, _vp, _c_i64, _vp]),
    "insite_gen_gram_workspace_bytes": (_c_size, [_c_i64, _c_i32, _c_i32, _c_i32]),
    "insite_gen_gram_f64": (_c_i32, [_vp, _c_i64, _c_i32, _c_i32, _vp, _c_i32, _vp, _c_i64, _c_i32, _vp, _c_i32, _vp,
                                     _c_i64, _vp, _c_i32, _c_i32, _c_f64, _vp, _vp, _vp, _c_size, _vp]),
    "insite_stlsq_wave64_f64": (_c_i32, [_vp, _vp, _c_i64, _c_i32, _c_f64, _c_f64, _c_i32, _c_i32, _vp, _vp, _vp,
                                         _vp]),
    "insite_rollout_poly_f64": (_c_i32, [_vp, _vp, _vp, _c_i64, _vp, _c_i64, _vp, _c_i32, _c_i64, _c_i32, _c_i32,
                                         _c_i32, _c_f64, _c_i32, _c_i32, _c_f64, _vp, _c_i64, _c_i32, _vp]),
}


def load(path: str | None = None):
    """Load (once) and return the ctypes handle; raises InsiteLibraryError if unavailable."""
    global _lib
    if path is None and _lib is not None:   # lock-free fast path once loaded
        return _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise InsiteLibraryError(
                f"{p} is missing: build the HIP extension first (python -c 'import __graft_entry__ as g; g.build()')")
        try:
            lib = ctypes.CDLL(p, mode=ctypes.RTLD_LOCAL)
        except OSError as e:  # pragma: no cover - environment specific
            raise InsiteLibraryError(f"cannot load {p}: {e}") from e
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        v = lib.insite_abi_version()
        if v != ABI_VERSION:
            raise InsiteLibraryError(f"ABI version mismatch: library {v}, bindings {ABI_VERSION}")
        if path is None:
            _lib = lib
        return lib


def check(fn_name: str, code: int):
    if code != INSITE_OK:
        msg = load().insite_strerror(code).decode()
        raise InsiteError(fn_name, code, msg)
