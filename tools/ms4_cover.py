"""Moment cover of the C3 Gram for gram_ms4_kernel (csrc/insite_ms.hip, INSITE_MS4_COVER).

The C3 library Theta (5 states x_1..x_5 + one binary treatment a, degree 2, interaction only: F = 22,
pysindy order; oracle/multistate_ref.py c3_library) makes the Gram G = sum Theta^T Theta (253 upper-triangle
entries) and B = sum Theta^T xdot (110).  Every G entry is a monomial moment sum z^g with z = (x, a); since a
is 0/1 (a^2 = a, exact), the 253 entries hold only 147 distinct moments (168 without the a^2 = a identity),
and B adds 110.  A 4 x 4 x 4 f64 MFMA block of operand groups U x V accumulates 16 moments u_m v_n.  The
round-1..4 layout (Theta | xdot in 7 column groups, blocks rg <= cg) issues 27 blocks = 432 cells per row
for 363 entries; this tool searches operand groups (each operand a product of <= 2 staged "pure" values
[1, x_1..x_5, a, xdot_1..xdot_5], i.e. one LDS read or two reads + one multiply) whose pairwise blocks cover
all 257 distinct moments with fewer blocks, then emits the tables the kernel and its finalize use.

    python tools/ms4_cover.py --search --groups 8 --iters 150000 --seed 1 --out sol.json [--init sol0.json]
    python tools/ms4_cover.py --emit sol.json          # -> csrc/ms4_cover_c3.inc (blocks by exact ILP)

Code-generation tool: not imported by the product; tests/test_ms4_cover.py checks its output independently.
"""
import argparse
import collections
import json
import math
import os
import random

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd", "csrc",
                   "ms4_cover_c3.inc")

S, NIN = 5, 1
NZ = S + NIN
A_POS = NZ            # staged position of the binary treatment a
NPURE = NZ + 1 + S    # staged pure values: [1, x_1..x_5, a, xdot_1..xdot_5]


def mono(*pos):
    """Monomial of staged positions (0 = the constant); a^2 = a."""
    c = collections.Counter(p for p in pos if p != 0)
    if c[A_POS] > 1:
        c[A_POS] = 1
    return tuple(sorted(c.items()))


# library columns in pysindy order (PolyCols<NZ, true>): 1; z_1..z_NZ; z_i z_k (i < k)
LIB = [(0, 0)] + [(i, 0) for i in range(1, NZ + 1)] + [(i, k) for i in range(1, NZ + 1) for k in range(i + 1, NZ + 1)]
F = len(LIB)
XD = list(range(NZ + 1, NPURE))  # staged positions of xdot_s


def entry_moments():
    """(kind, j, k) -> moment for every output entry: G[j][k] (full square) and B[j][s]."""
    out = {}
    for j in range(F):
        for k in range(F):
            out[("G", j, k)] = mono(*LIB[j], *LIB[k])
        for s in range(S):
            out[("B", j, s)] = mono(*LIB[j], XD[s])
    return out


ENTRIES = entry_moments()
NEED = sorted(set(ENTRIES.values()))
IDX = {m: i for i, m in enumerate(NEED)}
FULL = (1 << len(NEED)) - 1

# operand family: products of two staged values with at most one xdot factor
OPS = {}
for pa in range(NPURE):
    for pb in range(pa + 1):
        if pa in XD and pb in XD:
            continue
        m = mono(pa, pb)
        cost = 1 if pb == 0 else 2
        if m not in OPS or OPS[m][1] > cost:
            OPS[m] = ((pa, pb), cost)
if os.environ.get("MS4_COVER_TRIPLES"):  # search-only: operands of three staged factors (3 reads, 2 multiplies)
    for pa in range(1, NZ + 1):
        for pb in range(1, pa + 1):
            for pc in range(1, pb + 1):
                m = mono(pa, pb, pc)
                if m not in OPS:
                    OPS[m] = ((pa, pb, pc), 3)
OPL = list(OPS)
NO = len(OPL)


def _prod(u, v):
    fa = [p for p, e in OPL[u] for _ in range(e)]
    fb = [p for p, e in OPL[v] for _ in range(e)]
    return IDX.get(mono(*fa, *fb))


PT = [[_prod(u, v) for v in range(NO)] for u in range(NO)]


def block_bits(g, h):
    b = 0
    for u in g:
        for v in h:
            p = PT[u][v]
            if p is not None:
                b |= 1 << p
    return b


def candidates(groups):
    out = []
    for i in range(len(groups)):
        for j in range(i, len(groups)):
            b = block_bits(groups[i], groups[j])
            if b:
                out.append((b, i, j))
    return out


def greedy(groups):
    cands = candidates(groups)
    cov, chosen = 0, []
    while cov != FULL:
        best = max(cands, key=lambda c: bin(c[0] & ~cov).count("1"))
        if not best[0] & ~cov:
            return None, bin(FULL & ~cov).count("1")
        cov |= best[0]
        chosen.append(best)
    changed = True
    while changed:
        changed = False
        for c in list(chosen):
            rest = 0
            for d in chosen:
                if d is not c:
                    rest |= d[0]
            if rest == FULL:
                chosen.remove(c)
                changed = True
                break
    return chosen, 0


def exact(groups, time_limit=120):
    import numpy as np
    from scipy.optimize import Bounds, LinearConstraint, milp
    cands = candidates(groups)
    A = np.zeros((len(NEED), len(cands)))
    for c, (b, _, _) in enumerate(cands):
        for m in range(len(NEED)):
            if b >> m & 1:
                A[m, c] = 1
    res = milp(np.ones(len(cands)), constraints=LinearConstraint(A, 1, np.inf), integrality=np.ones(len(cands)),
               bounds=Bounds(0, 1), options={"time_limit": time_limit})
    if res.x is None:
        raise SystemExit("no cover")
    return [cands[c] for c in range(len(cands)) if res.x[c] > 0.5]


def gcost(groups):
    reads = muls = 0
    for g in groups:
        c = max(OPS[OPL[u]][1] for u in g)
        reads += c
        muls += c - 1
    return reads, muls


def score(groups, lam):
    ch, unc = greedy(groups)
    if ch is None:
        return 1000 + 10 * unc, None
    return len(ch) + lam * gcost(groups)[0], ch


def anneal(groups, iters, seed, lam, t0=0.6):
    rnd = random.Random(seed)
    ng = len(groups)
    s, ch = score(groups, lam)
    best = (s, [g[:] for g in groups], ch)
    for it in range(iters):
        temp = max(0.03, t0 * (1 - it / iters))
        if rnd.random() < 0.5:
            g, k = rnd.randrange(ng), rnd.randrange(4)
            old = groups[g][k]
            groups[g][k] = rnd.randrange(NO)

            def undo(g=g, k=k, old=old):
                groups[g][k] = old
        else:
            g, h, k, l = rnd.randrange(ng), rnd.randrange(ng), rnd.randrange(4), rnd.randrange(4)
            groups[g][k], groups[h][l] = groups[h][l], groups[g][k]

            def undo(g=g, h=h, k=k, l=l):
                groups[g][k], groups[h][l] = groups[h][l], groups[g][k]
        s2, ch2 = score(groups, lam)
        if s2 <= s or rnd.random() < math.exp((s - s2) / temp):
            s, ch = s2, ch2
            if s < best[0]:
                best = (s, [x[:] for x in groups], ch)
        else:
            undo()
    return best


def to_json(groups):
    return [[list(OPS[OPL[u]][0]) for u in g] for g in groups]


def from_json(gj):
    rev = {tuple(v[0]): m for m, v in OPS.items()}
    out = []
    for g in gj:
        row = []
        for pa, pb in g:
            m = mono(pa, pb)
            row.append(OPL.index(m))
        out.append(row)
    return out


def layout(groups, blocks):
    """Per-entry partial index t * 16 + 4 m + n (block t: U = groups[bu], V = groups[bv]); -1 never."""
    where = {}
    for t, (_, u, v) in enumerate(blocks):
        for m in range(4):
            for n in range(4):
                p = PT[groups[u][m]][groups[v][n]]
                if p is not None and p not in where:
                    where[p] = t * 16 + 4 * m + n
    qmap = []
    for key in [("G", j, k) for j in range(F) for k in range(F)] + [("B", j, s) for j in range(F) for s in range(S)]:
        q = where.get(IDX[ENTRIES[key]])
        assert q is not None, key
        qmap.append(q)
    return qmap


STRIDE = (4 * ((NPURE + 3) // 4)) | 1  # staged row stride (Ms4Z::STRIDE)


def _read_cycles(pos):
    """LDS cycles of one ds_read_b64 of slot positions pos[0..3] in the kernel's row pattern, averaged over the 4
    passes and the two 32-lane groups (1.0 = conflict-free; bank of dword a = a mod 64)."""
    tot = 0
    for r in range(4):
        for half in (0, 1):
            banks = collections.defaultdict(set)
            for lane in range(32 * half, 32 * half + 32):
                k, b = lane >> 4, (lane >> 2) & 3
                d = (32 * (k >> 1) + 4 * (4 * (k & 1) + b) + r) * STRIDE + pos[lane & 3]
                for w in (2 * d, 2 * d + 1):
                    banks[w % 64].add(d)
            tot += max(len(v) for v in banks.values())
    return tot / 8


def orient(ops, pi=None):
    """Per group, the slot order and (product groups) the factor order of each slot -- a product commutes --
    that minimise the group's reads' bank conflicts, the pure values staged at positions pi[v].
    Returns (ops in staged positions, slot permutation per group, LDS cycles per pass)."""
    import itertools
    pi = list(range(NPURE)) if pi is None else pi
    out, perms, tot = [], [], 0.0
    for g in ops:
        prod = any(pb for _, pb in g)
        best = None
        for perm in itertools.permutations(range(4)):
            for bits in range(16 if prod else 1):
                gg = [g[perm[i]] for i in range(4)]
                gg = [(pi[pb], pi[pa]) if bits >> i & 1 else (pi[pa], pi[pb]) for i, (pa, pb) in enumerate(gg)]
                c = _read_cycles([x[0] for x in gg]) + (_read_cycles([x[1] for x in gg]) if prod else 0)
                if best is None or c < best[0] - 1e-9:
                    best = (c, gg, perm)
        out.append(best[1])
        perms.append(best[2])
        tot += best[0]
    return out, perms, tot


def stage_order(ops, iters=3000, seed=1):
    """Staged position of every pure value (a permutation of the row) for conflict-free operand reads: swap
    hill-climb from the identity."""
    rnd = random.Random(seed)
    pi = list(range(NPURE))
    best = orient(ops, pi)[2]
    for _ in range(iters):
        if best <= sum(1 + any(pb for _, pb in g) for g in ops):
            break  # every read conflict-free
        i, j = rnd.randrange(NPURE), rnd.randrange(NPURE)
        pi[i], pi[j] = pi[j], pi[i]
        c = orient(ops, pi)[2]
        if c <= best:
            best = c
        else:
            pi[i], pi[j] = pi[j], pi[i]
    return pi


def emit(sol, path=INC):
    groups = from_json(sol["groups"])
    blocks = exact(groups)
    # order blocks by U group then V group (operands of one group stay live together)
    blocks.sort(key=lambda b: (b[1], b[2]))
    vops = [[OPS[OPL[u]][0] for u in g] for g in groups]
    prod = [int(any(pb for _, pb in g)) for g in vops]
    pi = stage_order(vops)
    ops, perms, conf = orient(vops, pi)
    groups = [[g[p[i]] for i in range(4)] for g, p in zip(groups, perms)]
    qmap = layout(groups, blocks)
    print(f"LDS cycles per pass of the operand reads: {conf:.1f}")
    reads, muls = gcost(groups)
    lines = [
        "// generated by tools/ms4_cover.py --emit (do not edit): moment cover of the C3 Gram (S = 5, one binary",
        f"// input, interaction-only degree 2, F = {F}) -- {len(groups)} operand groups, {len(blocks)} 4 x 4 x 4 f64 blocks "
        f"({len(blocks) * 16} cells) for {len(NEED)} distinct moments",
        f"// ({F * (F + 1) // 2} G entries + {F * S} B entries); per pass {reads} LDS reads, {muls} product groups.",
        f"constexpr int kMs4CoverNG = {len(groups)};",
        f"constexpr int kMs4CoverNB = {len(blocks)};",
        f"constexpr int kMs4CoverEntries = {len(qmap)};  // F * F (G, row-major) + F * S (B, row-major)",
        "// staged position of pure value v = [1, x_1..x_5, a, xdot_1..xdot_5][v] (a permutation of the row that",
        "// makes every operand read below bank-conflict-free)",
        "constexpr unsigned char kMs4CoverStage[" + str(NPURE) + "] = {" + ", ".join(str(p) for p in pi) + "};",
        "// staged positions of the two factors of slot i of group g (a pure operand's second factor is the 1.0)",
        "constexpr unsigned char kMs4CoverPA[kMs4CoverNG][4] = {"
        + ", ".join("{" + ", ".join(str(o[0]) for o in g) + "}" for g in ops) + "};",
        "constexpr unsigned char kMs4CoverPB[kMs4CoverNG][4] = {"
        + ", ".join("{" + ", ".join(str(o[1]) for o in g) + "}" for g in ops) + "};",
        "constexpr unsigned char kMs4CoverProd[kMs4CoverNG] = {" + ", ".join(map(str, prod))
        + "};  // group reads two factors",
        "// block t = U group kMs4CoverBU[t] (MFMA A) x V group kMs4CoverBV[t] (MFMA B)",
        "constexpr unsigned char kMs4CoverBU[kMs4CoverNB] = {" + ", ".join(str(b[1]) for b in blocks) + "};",
        "constexpr unsigned char kMs4CoverBV[kMs4CoverNB] = {" + ", ".join(str(b[2]) for b in blocks) + "};",
        "// output entry -> block partial index t * 16 + 4 m + n",
        "__constant__ unsigned short kMs4CoverMap[kMs4CoverEntries] = {",
    ]
    for i in range(0, len(qmap), 22):
        lines.append("    " + ", ".join(str(q) for q in qmap[i:i + 22]) + ",")
    lines.append("};")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    print(f"wrote {path}: {len(groups)} groups, {len(blocks)} blocks, reads {reads}, muls {muls}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--search", action="store_true")
    ap.add_argument("--groups", type=int, default=8)
    ap.add_argument("--iters", type=int, default=100000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--lam", type=float, default=0.03, help="weight of the per-pass LDS reads in the objective")
    ap.add_argument("--init", default=None)
    ap.add_argument("--out", default=None)
    ap.add_argument("--emit", default=None)
    args = ap.parse_args()
    print(f"F = {F}: {F * (F + 1) // 2} + {F * S} entries, {len(NEED)} distinct moments, {NO} operands")
    if args.search:
        rnd = random.Random(args.seed)
        groups = from_json(json.load(open(args.init))["groups"]) if args.init else []
        while len(groups) < args.groups:
            groups.append([rnd.randrange(NO) for _ in range(4)])
        s, groups, ch = anneal(groups, args.iters, args.seed, args.lam)
        blocks = exact(groups)
        print(f"blocks {len(blocks)} (greedy {None if ch is None else len(ch)}), reads/muls {gcost(groups)}")
        if args.out:
            json.dump({"groups": to_json(groups), "blocks": len(blocks)}, open(args.out, "w"), indent=1)
    if args.emit:
        emit(json.load(open(args.emit)))


if __name__ == "__main__":
    main()
