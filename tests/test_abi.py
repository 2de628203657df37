"""CPU tests of the C ABI (libinsite_hip.so) — no GPU and no compute launches.

The library is the drop-in boundary (include/insite_hip.h): it must load, export every symbol
the header declares, answer the host-side queries (version, error strings, library table,
workspace sizes) and reject invalid arguments before touching the device.  The product ops
must refuse host tensors (there is no CPU fallback).
"""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "insite_hip.h")


@pytest.fixture(scope="module")
def L():
    from insite_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build()
    return _lib.load()


def _header_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+char\s*\*|int32_t|size_t)\s+(insite_\w+)\s*\(", src, re.M)))


def _lib_exports():
    from insite_amd import _lib
    return _lib.EXPORTS


def test_header_declares_the_abi():
    fns = _header_functions()
    assert "insite_rollout_f64" in fns and "insite_sindy_fit_f64" in fns
    assert len(fns) == 43 and set(fns) == set(_lib_exports())


def test_library_exports_every_header_symbol(L):
    from insite_amd import _lib
    for name in _header_functions():
        assert hasattr(L, name), name
    assert sorted(_lib.EXPORTS) == _header_functions()


def test_nm_shows_c_linkage():
    """The entry points are unmangled extern "C" symbols of the shared object."""
    import subprocess
    from insite_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    syms = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    for name in _header_functions():
        assert name in syms, name


def test_version_and_strerror(L):
    from insite_amd import _lib
    assert L.insite_abi_version() == _lib.ABI_VERSION == 9
    assert L.insite_strerror(0) == b"ok"
    for code in (-1, -2, -3, -4):
        s = L.insite_strerror(code)
        assert s and s != b"ok"


def test_header_constants_match_bindings():
    from insite_amd import _lib
    src = open(HEADER).read()

    def const(name):
        return int(re.search(rf"#define {name} \(?(-?\d+)\)?", src).group(1))

    assert const("INSITE_OK") == _lib.INSITE_OK
    assert (const("INSITE_FD_SMOOTHED4"), const("INSITE_FD_ORDER4"), const("INSITE_FD_ORDER1"),
            const("INSITE_FD_SMOOTHED1")) == (_lib.FD_SMOOTHED4, _lib.FD_ORDER4, _lib.FD_ORDER1, _lib.FD_SMOOTHED1)
    assert (const("INSITE_METHOD_EULER"), const("INSITE_METHOD_RK4")) == (_lib.METHOD_EULER, _lib.METHOD_RK4)
    assert (const("INSITE_LAYOUT_PATIENT_MAJOR"), const("INSITE_LAYOUT_TIME_MAJOR"),
            const("INSITE_LAYOUT_TIME_MAJOR_BITS")) == \
        (_lib.LAYOUT_PATIENT_MAJOR, _lib.LAYOUT_TIME_MAJOR, _lib.LAYOUT_TIME_MAJOR_BITS)
    assert (const("INSITE_MAX_TERMS"), const("INSITE_MAX_STATICS"), const("INSITE_MAX_ARMS")) == \
        (_lib.MAX_TERMS, _lib.MAX_STATICS, _lib.MAX_ARMS)


@pytest.mark.parametrize("n_statics,degree,io", [(2, 2, True), (1, 2, False), (3, 2, True), (0, 1, True),
                                                 (2, 1, True), (1, 3, False)])
def test_poly_library_native_matches_oracle(L, n_statics, degree, io):
    from oracle import insite_ref as R
    from insite_amd import ops
    from insite_amd.library import polynomial_library
    native = ops.poly_library_native(n_statics, degree, io)
    ref = R.poly_library(1 + n_statics, degree, io)
    np.testing.assert_array_equal(native, ref)
    np.testing.assert_array_equal(polynomial_library(n_statics, degree, io).exps, ref)


def test_poly_library_names():
    from insite_amd.library import polynomial_library
    lib = polynomial_library(2, 2, True)
    assert lib.get_feature_names() == ["1", "x0", "u0", "u1", "x0 u0", "x0 u1", "u0 u1"]
    assert lib.n_terms == 7 and lib.n_statics == 2 and lib.state_degree == 1


def test_poly_library_errors(L):
    buf = np.zeros((4, 3), np.int8)
    n = ctypes.c_int32(0)
    # too small an output table
    st = L.insite_poly_library(2, 2, 1, buf.ctypes.data_as(ctypes.c_void_p), 4, ctypes.byref(n))
    assert st < 0
    st = L.insite_poly_library(-1, 2, 1, buf.ctypes.data_as(ctypes.c_void_p), 4, ctypes.byref(n))
    assert st == -1


def test_workspace_queries(L):
    a = L.insite_gram_workspace_bytes(1000, 2, 7)
    b = L.insite_gram_workspace_bytes(10_000_000, 2, 7)
    assert 0 < a <= b
    assert L.insite_masked_sse_workspace_bytes(100, 10) > 0
    assert L.insite_masked_sse_workspace_bytes(-1, 10) == 0


def test_invalid_arguments_rejected_without_device(L):
    """Argument validation happens before any HIP call (these run on a GPU-less host)."""
    from insite_amd import _lib
    nul = ctypes.c_void_p(0)
    exps = np.zeros((7, 3), np.int8)
    ep = exps.ctypes.data_as(ctypes.c_void_p)
    # rollout: negative rows, bad layout, too many arms, substeps < 1; zero-size is a no-op success
    assert L.insite_rollout_f64(nul, nul, nul, 4, nul, 0, ep, 7, -1, 4, 2, 2, 0.1, 1, 1, 1e-3, nul, 4, 0, nul) == -1
    assert L.insite_rollout_f64(nul, nul, nul, 4, nul, 0, ep, 7, 8, 4, 2, 2, 0.1, 1, 1, 1e-3, nul, 4, 7, nul) == -1
    assert L.insite_rollout_f64(nul, nul, nul, 4, nul, 0, ep, 7, 8, 4, 2, 9, 0.1, 1, 1, 1e-3, nul, 4, 0, nul) == -1
    assert L.insite_rollout_f64(nul, nul, nul, 4, nul, 0, ep, 7, 8, 4, 2, 2, 0.1, 1, 0, 1e-3, nul, 4, 0, nul) == -1
    assert L.insite_rollout_f64(nul, nul, nul, 4, nul, 0, ep, 7, 0, 4, 2, 2, 0.1, 1, 1, 1e-3, nul, 4, 0, nul) == 0
    # time-major leading dimension must cover the patients
    assert L.insite_rollout_f64(nul, nul, nul, 4, nul, 0, ep, 7, 8, 4, 2, 2, 0.1, 1, 1, 1e-3, nul, 8,
                                _lib.LAYOUT_TIME_MAJOR, nul) == -1
    # bit-packed arms: at most 2 arms; leading dimension in words must cover the patients
    assert L.insite_rollout_f64(nul, nul, nul, 1, nul, 0, ep, 7, 64, 4, 2, 3, 0.1, 1, 1, 1e-3, nul, 64,
                                _lib.LAYOUT_TIME_MAJOR_BITS, nul) == -1
    assert L.insite_rollout_f64(nul, nul, nul, 1, nul, 0, ep, 7, 65, 4, 2, 2, 0.1, 1, 1, 1e-3, nul, 65,
                                _lib.LAYOUT_TIME_MAJOR_BITS, nul) == -1
    # stlsq: negative systems / threshold; n_sys = 0 is a no-op
    assert L.insite_stlsq_f64(nul, nul, -1, 7, 0.1, 0.5, 100, 1, nul, nul, nul, nul) == -1
    assert L.insite_stlsq_f64(nul, nul, 4, 7, -0.1, 0.5, 100, 1, nul, nul, nul, nul) == -1
    assert L.insite_stlsq_f64(nul, nul, 0, 7, 0.1, 0.5, 100, 1, nul, nul, nul, nul) == 0
    # gram: null outputs, unsupported derivative kind, short workspace
    assert L.insite_gram_f64(nul, 60, 0, 60, nul, nul, nul, 10, 2, 2, ep, 7, 0, 0.1, nul, nul, nul, 0, nul) == -1
    g = (ctypes.c_double * 98)()
    bb = (ctypes.c_double * 14)()
    x = (ctypes.c_double * 600)()
    assert L.insite_gram_f64(x, 60, 0, 60, x, x, x, 10, 2, 2, ep, 7, _lib.FD_ORDER1, 0.1, g, bb, nul, 0, nul) == -2
    assert L.insite_gram_f64(x, 60, 0, 60, x, x, x, 10, 2, 2, ep, 7, 0, 0.1, g, bb, nul, 0, nul) == -3
    # bad layout; patient-major n_steps beyond ldx; time-major ldx below the patient count
    assert L.insite_gram_f64(x, 60, 5, 60, x, x, x, 10, 2, 2, ep, 7, 0, 0.1, g, bb, nul, 0, nul) == -1
    assert L.insite_gram_f64(x, 60, 0, 61, x, x, x, 10, 2, 2, ep, 7, 0, 0.1, g, bb, nul, 0, nul) == -1
    assert L.insite_gram_f64(x, 9, 1, 60, x, x, x, 10, 2, 2, ep, 7, 0, 0.1, g, bb, nul, 0, nul) == -1
    # library with a state exponent > 1 is outside this ABI version
    e2 = np.zeros((7, 3), np.int8)
    e2[1, 0] = 2
    assert L.insite_gram_f64(x, 60, 0, 60, x, x, x, 10, 2, 2, e2.ctypes.data_as(ctypes.c_void_p), 7, 0, 0.1, g, bb,
                             nul, 0, nul) == -2
    # treatment-segment discovery (F4): FD kinds of the cancer_sim / EQ_5 path only; arm leading dim;
    # short workspace; the fit validates its STLSQ arguments first
    o1, s1 = _lib.FD_ORDER1, _lib.FD_SMOOTHED1
    seg = L.insite_gram_segments_f64
    assert seg(x, 60, x, 59, 0, 60, x, x, 10, 2, 4, ep, 7, 0, 0.1, g, bb, nul, 0, nul) == -2        # smoothed4
    assert seg(x, 60, x, 58, 0, 60, x, x, 10, 2, 4, ep, 7, o1, 0.1, g, bb, nul, 0, nul) == -1       # ld_arm < T-1
    assert seg(x, 60, x, 59, 3, 60, x, x, 10, 2, 4, ep, 7, o1, 0.1, g, bb, nul, 0, nul) == -1       # layout
    assert seg(x, 9, x, 10, 1, 60, x, x, 10, 2, 4, ep, 7, o1, 0.1, g, bb, nul, 0, nul) == -1        # TM ldx < N
    assert seg(x, 60, x, 59, 0, 60, x, x, 10, 2, 5, ep, 7, s1, 0.1, g, bb, nul, 0, nul) == -1       # 5 arms
    assert seg(x, 60, x, 59, 0, 60, x, x, 10, 2, 4, ep, 7, s1, 0.1, g, bb, nul, 0, nul) == -3       # workspace
    assert L.insite_sindy_fit_segments_f64(x, 60, x, 59, 0, 60, x, x, 10, 2, 4, ep, 7, o1, 0.1, -1.0, 0.5, 100, 1,
                                           g, bb, g, nul, nul, nul, 0, nul) == -1
    assert 0 < L.insite_gram_segments_workspace_bytes(1000, 4, 7) <= L.insite_gram_segments_workspace_bytes(10**7, 4, 7)


def test_ops_refuse_host_tensors(L):
    """No CPU fallback: host tensors raise instead of silently computing elsewhere."""
    import torch
    from insite_amd import ops
    from insite_amd.library import polynomial_library
    lib = polynomial_library(2, 2, True)
    x = torch.zeros((4, 10), dtype=torch.float64)
    with pytest.raises(ValueError, match="device tensor"):
        ops.gram(x, torch.zeros((4, 2), dtype=torch.float64), torch.zeros(4, dtype=torch.int8),
                 torch.full((4,), 8, dtype=torch.int32), 0.1, lib)
    with pytest.raises(ValueError, match="device tensor"):
        ops.rollout(torch.zeros(4, dtype=torch.float64), torch.zeros((4, 2), dtype=torch.float64),
                    torch.zeros((4, 10), dtype=torch.int8), torch.zeros((2, 7), dtype=torch.float64), lib, 0.1)
    with pytest.raises(ValueError, match="device tensor"):
        ops.stlsq(torch.eye(7, dtype=torch.float64)[None], torch.zeros((1, 7), dtype=torch.float64), 0.1, 0.5)
    with pytest.raises(ValueError, match="device tensor"):
        ops.refine_prepare(torch.zeros((4, 10), dtype=torch.float64), torch.zeros((4, 10), dtype=torch.int8))
    with pytest.raises(ValueError, match="device tensor"):
        ops.refine_finish(torch.zeros((10, 4), dtype=torch.float64), None, 4)


def test_missing_library_fails_loudly(tmp_path):
    from insite_amd import _lib
    with pytest.raises(_lib.InsiteLibraryError):
        _lib.load(str(tmp_path / "nope.so"))


def test_product_package_does_not_import_oracle():
    """The product path never routes through the CPU oracle."""
    pkg = os.path.join(ROOT, "ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".hip", ".cpp", ".h")):
                src = open(os.path.join(dp, f)).read()
                assert "oracle" not in re.sub(r"#.*|//.*", "", src).replace("oracle/", ""), f


def test_pack_arm_bits_roundtrip():
    import torch
    from insite_amd import ops
    g = torch.Generator().manual_seed(0)
    for N in (1, 31, 32, 33, 100, 257):
        a = torch.randint(0, 2, (7, N + 3), generator=g, dtype=torch.int64).to(torch.int8)
        w = ops.pack_arm_bits(a, N)
        assert w.shape == (7, (N + 31) // 32) and w.dtype == torch.int32
        u = w.to(torch.int64) & 0xFFFFFFFF
        bits = (u[:, torch.arange(N) // 32] >> (torch.arange(N) % 32)) & 1
        assert torch.equal(bits.to(torch.int8), a[:, :N])
    with pytest.raises(ValueError):
        ops.pack_arm_bits(torch.full((2, 4), 2, dtype=torch.int8))


def test_deferred_workspace_holds_two_slots_and_the_claim_area():
    """insite_fit_rollout_deferred_workspace_bytes = the 4-KiB claim areas at offset 0 (the claimed gram tail's nine
    128-B head / done lines, then the claimed rollout tail's eight; their place does not move with the cohort size) +
    two discovery slots (insite_hip.h)."""
    from insite_amd import _lib
    L = _lib.load()
    for n in (1, 1000, 100_000, 1_000_000):
        assert L.insite_fit_rollout_deferred_workspace_bytes(n, 2, 7) == 2 * L.insite_gram_workspace_bytes(n, 2, 7) + 4096
