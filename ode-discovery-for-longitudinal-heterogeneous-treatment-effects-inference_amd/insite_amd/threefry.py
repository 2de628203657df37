"""jax.random's default PRNG (Threefry-2x32) on the device, as the reference drew its PK/PD cohorts.

The reference seeds every subset with ``jax.random.PRNGKey(seed)`` and derives each draw with
``key, subkey = jax.random.split(key)`` (``libs_m/ct/src/data/pkpd/dataset.py:52-54``;
``pkpd_simulation.py:117-197, 233-236, 290-291``), under ``jax_enable_x64`` (``pkpd_simulation.py:13``) and
the jax 0.4.x defaults of its 2023 logs (``jax_threefry_partitionable`` off).  The random words come from
the HIP kernel ``insite_threefry2x32_iota_u32`` (``csrc/insite_rng.hip``: ``threefry_2x32(key,
iota(n))``); the transforms follow jax's published algorithms on torch device tensors:

* ``split(key, num)``: words ``threefry_2x32(key, iota(2 num))`` as ``num`` key pairs;
* ``random_bits(key, 64, shape)``: ``2 size`` words, ``(first half << 32) | second half``;
* ``uniform``: mantissa fill ``bitcast((bits >> 12) | 0x3FF0...) - 1``, then ``max(lo, u (hi - lo) + lo)``;
* ``normal``: ``sqrt(2) erfinv(uniform(nextafter(-1, 0), 1))`` (torch's float64 erfinv: a few ulp from
  XLA's polynomial, far below every tolerance it feeds);
* ``permutation``: ``ceil(3 ln n / ln(2^32 - 1))`` rounds of (split, 32-bit keys, stable sort).

Keys are (k0, k1) pairs of host ints (two words read back per split: the key schedule, not the data);
all bulk words are produced and transformed on the device.  Pinned on the GPU against the Random123
known-answer vectors and the numpy restatement of jax.random (tests/test_gpu_threefry.py), and end to end by
``run.py`` reproducing the published EQ_4 runs (tests/test_gpu_run_reference.py).
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib


def _words(key, n: int, device) -> torch.Tensor:
    """threefry_2x32(key, iota(n)) as int64 values in [0, 2^32) on ``device``."""
    out = torch.empty((max(int(n), 1),), dtype=torch.int32, device=device)
    if n > 0:
        st = _lib.load().insite_threefry2x32_iota_u32(ctypes.c_uint32(int(key[0]) & 0xFFFFFFFF),
                                                       ctypes.c_uint32(int(key[1]) & 0xFFFFFFFF), int(n),
                                                       ctypes.c_void_p(out.data_ptr()),
                                                       ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream))
        _lib.check("insite_threefry2x32_iota_u32", st)
    return out[:n].to(torch.int64) & 0xFFFFFFFF


def prng_key(seed: int):
    s = int(seed)
    return ((s >> 32) & 0xFFFFFFFF, s & 0xFFFFFFFF)


def split(key, num: int, device) -> list:
    w = _words(key, 2 * int(num), device).cpu().tolist()
    return [(w[2 * i], w[2 * i + 1]) for i in range(int(num))]


def random_bits(key, bit_width: int, shape, device) -> torch.Tensor:
    shape = tuple(int(s) for s in shape)
    size = math.prod(shape) if shape else 1
    if bit_width == 32:
        return _words(key, size, device).reshape(shape)
    if bit_width == 64:
        w = _words(key, 2 * size, device)
        return ((w[:size] << 32) | w[size:]).reshape(shape)      # uint64 bits held in int64
    raise NotImplementedError(bit_width)


def uniform(key, shape, device, minval: float = 0.0, maxval: float = 1.0) -> torch.Tensor:
    bits = random_bits(key, 64, shape, device)
    fb = ((bits >> 12) & ((1 << 52) - 1)) | 0x3FF0000000000000
    floats = fb.view(torch.float64) - 1.0
    lo = torch.tensor(float(minval), dtype=torch.float64, device=device)
    return torch.maximum(lo, floats * (float(maxval) - float(minval)) + float(minval))


def normal(key, shape, device) -> torch.Tensor:
    lo = math.nextafter(-1.0, 0.0)
    return math.sqrt(2.0) * torch.erfinv(uniform(key, shape, device, lo, 1.0))


def permutation(key, n: int, device) -> torch.Tensor:
    x = torch.arange(int(n), device=device)
    rounds = int(math.ceil(3 * math.log(max(1, int(n))) / math.log(0xFFFFFFFF)))
    for _ in range(rounds):
        key, sub = split(key, 2, device)
        keys = random_bits(sub, 32, (int(n),), device)
        x = x[torch.sort(keys, stable=True).indices]
    return x


class Stream:
    """A key threaded through the reference's ``key, subkey = split(key)`` pattern: every draw splits the
    current key and draws from the subkey (the interface of insite_amd.pkpd's generators)."""

    def __init__(self, key, device):
        self.key = (int(key[0]), int(key[1]))
        self.dev = torch.device(device)

    def _sub(self):
        self.key, sub = split(self.key, 2, self.dev)
        return sub

    def normal(self, *shape):
        return normal(self._sub(), shape, self.dev)

    def uniform(self, *shape, lo: float = 0.0, hi: float = 1.0):
        return uniform(self._sub(), shape, self.dev, lo, hi)

    def permutation(self, n: int):
        return permutation(self._sub(), n, self.dev)

    def split_first(self, num: int):
        """``key = split(key, num)[0]`` (pkpd_simulation.py:616: ``key, *subkeys = split(key, n + 1)``)."""
        w = _words(self.key, 2 * int(num), self.dev)[:2].cpu().tolist()
        self.key = (w[0], w[1])


def subset_streams(seed: int, device):
    """dataset.py:52-54 / 64-71: key = PRNGKey(seed); key, k_params = split(key); key, k_sim = split(key)."""
    key = prng_key(seed)
    key, kp = split(key, 2, device)
    key, ks = split(key, 2, device)
    return Stream(kp, device), Stream(ks, device)
