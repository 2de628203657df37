"""The C3 moment cover table (csrc/ms4_cover_c3.inc, emitted by tools/ms4_cover.py) checked independently of
the tool that made it: every G / B entry of the C3 library must map to a block cell whose two operands multiply
to the entry's own monomial (a is the binary treatment: a^2 = a), and the table must be what the kernel assumes
(factor positions inside the staged row, blocks over existing groups, fewer blocks than the column-group form)."""
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd", "csrc",
                   "ms4_cover_c3.inc")
S, NIN = 5, 1
NZ = S + NIN
NPURE = NZ + 1 + S  # staged [1, x_1..x_5, a, xdot_1..xdot_5]


def _arr(text, name):
    m = re.search(name + r"(?:\[[^\]]*\])+\s*=\s*\{(.*?)\};", text, re.S)
    return [int(v) for v in re.findall(r"\d+", m.group(1))]


def _const(text, name):
    return int(re.search(r"constexpr int " + name + r"\s*=\s*(\d+)", text).group(1))


def _table():
    text = open(INC).read()
    ng, nb = _const(text, "kMs4CoverNG"), _const(text, "kMs4CoverNB")
    pa = np.array(_arr(text, "kMs4CoverPA")).reshape(ng, 4)
    pb = np.array(_arr(text, "kMs4CoverPB")).reshape(ng, 4)
    bu, bv = _arr(text, "kMs4CoverBU"), _arr(text, "kMs4CoverBV")
    qmap = _arr(text, "kMs4CoverMap")
    stage = _arr(text, "kMs4CoverStage")
    assert sorted(stage) == list(range(NPURE))
    inv = np.argsort(stage)  # staged position -> pure value
    prod = _arr(text, "kMs4CoverProd")
    for g in range(ng):  # a pure group's second factors are all the staged 1.0
        assert prod[g] or all(pb[g, i] == stage[0] for i in range(4))
    return ng, nb, inv[pa], inv[pb], bu, bv, qmap


def _staged_exps(pos):
    """Exponent vector over [x_1..x_5, a, xdot_1..xdot_5] of staged position pos (0 = the constant)."""
    e = np.zeros(NZ + S, np.int64)
    if pos:
        e[pos - 1] = 1
    return e


def _reduce(e):
    e = e.copy()
    e[NZ - 1] = min(e[NZ - 1], 1)  # binary treatment
    return tuple(e)


def test_cover_table_maps_every_entry_to_its_monomial():
    from insite_amd.multistate import ms_library
    lib = ms_library(S, NIN, True)
    E = lib.exps.astype(np.int64)  # [F, S + NIN] over (x, a)
    F = E.shape[0]
    ng, nb, pa, pb, bu, bv, qmap = _table()
    assert len(qmap) == F * F + F * S and len(bu) == len(bv) == nb
    assert pa.max() < NPURE and pb.max() < NPURE and max(bu + bv) < ng

    def operand(g, i):
        return _staged_exps(pa[g, i]) + _staged_exps(pb[g, i])

    def cell(q):
        t, m, n = q // 16, (q % 16) // 4, q % 4
        assert t < nb
        return _reduce(operand(bu[t], m) + operand(bv[t], n))

    lib_e = [np.concatenate([E[j], np.zeros(S, np.int64)]) for j in range(F)]
    for j in range(F):
        for k in range(F):
            assert cell(qmap[j * F + k]) == _reduce(lib_e[j] + lib_e[k]), ("G", j, k)
        for s in range(S):
            xd = np.zeros(NZ + S, np.int64)
            xd[NZ + s] = 1
            assert cell(qmap[F * F + j * S + s]) == _reduce(lib_e[j] + xd), ("B", j, s)
    # symmetric G entries read one partial (the finalize writes bitwise-equal halves)
    for j in range(F):
        for k in range(F):
            assert qmap[j * F + k] == qmap[k * F + j]


def test_cover_operands_are_single_products_without_xdot_squares():
    ng, nb, pa, pb, bu, bv, qmap = _table()
    xd = set(range(NZ + 1, NPURE))
    for g in range(ng):
        for i in range(4):
            assert not (pa[g, i] in xd and pb[g, i] in xd)
    # fewer MFMA blocks than the Theta | xdot column groups (27 for F = 22, S = 5)
    assert nb < 27
