"""jax_prng — numpy restatement of JAX's default PRNG (threefry2x32) as the reference used it.

TEST INFRASTRUCTURE ONLY (oracle/): imported by ``tests/`` and the oracle's reference-cohort
builder (``oracle/ref_cohort.py``), never by the product package.

Why: the reference draws every PK/PD cohort with ``jax.random`` (``PRNGKey(seed)`` per subset,
``libs_m/ct/src/data/pkpd/dataset.py:52-54``; ``split`` / ``normal`` / ``uniform`` /
``permutation`` in ``pkpd_simulation.py:117-122,181-182,196-197,233-236,290-291``), and its
published logs hold 16-digit discovered coefficients for exactly those cohorts
(``results/2_main_table/final_with_insite.txt:126,154,182,210``).  Reproducing the draws bit for
bit lets the oracle be pinned against reference-held outputs.

Third-party dependency restated: **jax / jaxlib** (absent here and not vendored; unpinned in
``setup/requirements.txt``).  The reference's logs are dated 2023-05 (``final_with_insite.txt:1``),
i.e. the jax 0.4.x line, where ``jax_threefry_partitionable`` defaulted to False (the flag flipped
in jax 0.5.0), ``jax_enable_x64`` is on (``pkpd_simulation.py:13``) and the default PRNG is
threefry2x32.  Published algorithm restated (jax/_src/prng.py, jax/_src/random.py of that line):

* ``threefry2x32``: Threefry-2x32 with 20 rounds, rotations (13,15,26,6)/(17,29,16,24), key
  schedule (k0, k1, k0^k1^0x1BD11BDA) injected every 4 rounds with the round counter added to the
  second word (Salmon et al., "Parallel random numbers: as easy as 1, 2, 3", SC'11).
* ``threefry_2x32(key, count)``: the flat count array (padded with one 0 if odd) is split in two
  halves x0 | x1, hashed pairwise, and the two output words are concatenated y0 | y1.
* ``PRNGKey(seed)``: [seed >> 32, seed & 0xFFFFFFFF] (uint32 pair).
* ``split(key, num)``: ``threefry_2x32(key, iota(2*num)).reshape(num, 2)``.
* ``_random_bits(key, bits, shape)``: ``threefry_2x32(key, iota(ceil(bits*size/32)))``; for 64
  bits the output halves are (hi | lo) = (first half << 32) | second half.
* ``uniform(key, shape, f64, lo, hi)``: mantissa trick ``bitcast((bits >> 12) | 0x3FF0...) - 1``,
  then ``max(lo, u*(hi-lo)+lo)``.
* ``normal``: ``sqrt(2) * erfinv(uniform(key, shape, nextafter(-1, 0), 1))``.  XLA's f64
  ``ErfInv`` is a polynomial (Giles 2010); ``scipy.special.erfinv`` is used here, which agrees to
  a few ulp — far below the 1e-8 coefficient tolerance the pin uses (the cohorts' noise draws are
  0.01·N(0,1), so an ulp of the normal is ~1e-18 absolute in the data).
* ``permutation(key, x, independent=True)`` on 1-D x: ``_shuffle`` — ``ceil(3 ln n / ln(2^32-1))``
  rounds of (split, 32-bit sort keys, stable key/value sort).

Pinned by the Random123 known-answer vectors for Threefry-2x32-20 and by the jax documentation's
``split(PRNGKey(0))`` value (tests/test_jax_prng.py), then end to end by reproducing the published
EQ_4 coefficients (tests/test_reference_cohort.py).
"""
from __future__ import annotations

import math

import numpy as np
from scipy.special import erfinv

_M32 = np.uint64(0xFFFFFFFF)
_ROT = ((13, 15, 26, 6), (17, 29, 16, 24))


def _rotl(v: np.ndarray, r: int) -> np.ndarray:
    return ((v << np.uint32(r)) | (v >> np.uint32(32 - r))).astype(np.uint32)


def threefry2x32_block(k0, k1, x0: np.ndarray, x1: np.ndarray):
    """Threefry-2x32-20 on counter pairs (x0, x1) under key (k0, k1); uint32 arrays."""
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    ks = (k0, k1, np.uint32(k0 ^ k1 ^ np.uint32(0x1BD11BDA)))
    with np.errstate(over="ignore"):
        a = (np.asarray(x0, dtype=np.uint32) + ks[0]).astype(np.uint32)
        b = (np.asarray(x1, dtype=np.uint32) + ks[1]).astype(np.uint32)
        for g in range(5):
            for r in _ROT[g % 2]:
                a = (a + b).astype(np.uint32)
                b = _rotl(b, r) ^ a
            a = (a + ks[(g + 1) % 3]).astype(np.uint32)
            b = (b + ks[(g + 2) % 3] + np.uint32(g + 1)).astype(np.uint32)
    return a, b


def threefry_2x32(key, count: np.ndarray) -> np.ndarray:
    """``jax.prng.threefry_2x32(keypair, count)``: hash a flat uint32 count array."""
    c = np.asarray(count, dtype=np.uint32).ravel()
    odd = c.size % 2
    if odd:
        c = np.concatenate([c, np.zeros(1, dtype=np.uint32)])
    h = c.size // 2
    y0, y1 = threefry2x32_block(key[0], key[1], c[:h], c[h:])
    out = np.concatenate([y0, y1])
    return out[:-1] if odd else out


def PRNGKey(seed: int) -> np.ndarray:
    s = int(seed)
    return np.array([(s >> 32) & 0xFFFFFFFF, s & 0xFFFFFFFF], dtype=np.uint32)


def split(key, num: int = 2) -> np.ndarray:
    return threefry_2x32(key, np.arange(2 * num, dtype=np.uint32)).reshape(num, 2)


def random_bits(key, bit_width: int, shape) -> np.ndarray:
    shape = tuple(shape)
    size = int(np.prod(shape)) if shape else 1
    max_count, r = divmod(bit_width * size, 32)
    max_count += 1 if r else 0
    if max_count >= 0xFFFFFFFF:
        raise NotImplementedError("more than 2^32-1 words per draw")
    bits = threefry_2x32(key, np.arange(max_count, dtype=np.uint32))
    if bit_width == 32:
        return bits.reshape(shape)
    if bit_width == 64:
        hi, lo = bits[:size].astype(np.uint64), bits[size:].astype(np.uint64)
        return ((hi << np.uint64(32)) | lo).reshape(shape)
    raise NotImplementedError(bit_width)


def uniform(key, shape=(), minval=0.0, maxval=1.0) -> np.ndarray:
    """float64 ``jax.random.uniform`` (x64 mode)."""
    bits = random_bits(key, 64, shape)
    fb = (bits >> np.uint64(64 - 52)) | np.uint64(0x3FF0000000000000)
    floats = fb.view(np.float64) - 1.0
    lo, hi = np.float64(minval), np.float64(maxval)
    return np.maximum(lo, floats * (hi - lo) + lo).reshape(shape)


def normal(key, shape=()) -> np.ndarray:
    """float64 ``jax.random.normal``."""
    lo = np.nextafter(np.float64(-1.0), np.float64(0.0))
    u = uniform(key, shape, lo, 1.0)
    return (np.float64(np.sqrt(2.0)) * erfinv(u)).reshape(shape)


def permutation(key, x) -> np.ndarray:
    """``jax.random.permutation(key, x, independent=True)`` for a 1-D array x (``_shuffle``)."""
    x = np.asarray(x)
    n = x.size
    rounds = int(math.ceil(3 * math.log(max(1, n)) / math.log(0xFFFFFFFF)))
    for _ in range(rounds):
        key, sub = split(key)
        sort_keys = random_bits(sub, 32, x.shape)
        x = x[np.argsort(sort_keys, kind="stable")]
    return x
