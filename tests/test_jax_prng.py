"""The JAX threefry2x32 restatement (oracle/jax_prng.py) against published known answers.

* Random123 known-answer vectors for Threefry-2x32-20 (Salmon et al., SC'11; the same vectors
  jax's own tests use);
* ``jax.random.split(jax.random.PRNGKey(0))`` = [[4146024105, 967050713], [2718843009, 1272950319]]
  (jax documentation, "Pseudo random numbers in JAX").
The end-to-end pin — the reference's logged cohorts reproduced — is tests/test_reference_cohort.py.
"""
import numpy as np
import pytest

from oracle import jax_prng as J


@pytest.mark.parametrize("key,ctr,out", [
    ((0x00000000, 0x00000000), (0x00000000, 0x00000000), (0x6B200159, 0x99BA4EFE)),
    ((0xFFFFFFFF, 0xFFFFFFFF), (0xFFFFFFFF, 0xFFFFFFFF), (0x1CB996FC, 0xBB002BE7)),
    ((0x13198A2E, 0x03707344), (0x243F6A88, 0x85A308D3), (0xC4923A9C, 0x483DF7A0)),
])
def test_threefry2x32_random123_kat(key, ctr, out):
    a, b = J.threefry2x32_block(key[0], key[1], np.array([ctr[0]], np.uint32), np.array([ctr[1]], np.uint32))
    assert (int(a[0]), int(b[0])) == out


def test_split_prngkey0_documented_value():
    assert J.PRNGKey(0).tolist() == [0, 0]
    assert J.split(J.PRNGKey(0)).tolist() == [[4146024105, 967050713], [2718843009, 1272950319]]


def test_odd_count_padding_and_shapes():
    k = J.PRNGKey(7)
    b3 = J.threefry_2x32(k, np.arange(3, dtype=np.uint32))
    b4 = J.threefry_2x32(k, np.arange(4, dtype=np.uint32))
    assert b3.shape == (3,) and b4.shape == (4,)
    # odd counts hash [0,1,2,0] split as (0,1)|(2,0): element 0 pairs with 2, not with 3
    y0, y1 = J.threefry2x32_block(k[0], k[1], np.array([0, 1], np.uint32), np.array([2, 0], np.uint32))
    assert b3.tolist() == [int(y0[0]), int(y0[1]), int(y1[0])]
    assert J.random_bits(k, 64, (2, 3)).shape == (2, 3)


def test_uniform_normal_permutation_properties():
    k = J.PRNGKey(3)
    u = J.uniform(k, (200_000,), 1.0, 50.0)
    assert u.min() >= 1.0 and u.max() < 50.0 and abs(u.mean() - 25.5) < 0.2
    z = J.normal(k, (200_000,))
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1.0) < 0.01
    p = J.permutation(k, np.arange(1000))
    assert sorted(p.tolist()) == list(range(1000)) and p.tolist() != list(range(1000))
    # uniform uses the top 52 bits of the 64-bit draw: values are exact multiples of 2^-52 in [0, 1)
    u01 = J.uniform(k, (1000,))
    assert np.all(np.ldexp(u01, 52) == np.floor(np.ldexp(u01, 52)))
