"""The XCD-major rank of the deferred step's rollout blocks (csrc/insite_hip.hip xcd_count / xcd_rank,
INSITE_DEF_XCD), restated: for the blocks [lo, hi) it must be a bijection onto [0, hi - lo) (every rollout wave
gets one range, none twice) and give the blocks of one XCD (b % 8) consecutive ranks in block order.  CPU only;
the kernel's outputs are checked on the GPU (tests/test_gpu_deferred.py, test_gpu_fused.py)."""
import pytest

K_XCDS = 8


def xcd_count(n, x):
    return (n + K_XCDS - 1 - x) // K_XCDS


def xcd_rank(b, lo, hi):
    x = b % K_XCDS
    r = xcd_count(b, x) - xcd_count(lo, x)
    for q in range(x):
        r += xcd_count(hi, q) - xcd_count(lo, q)
    return r


@pytest.mark.parametrize("lo", [0, 1, 5, 257, 258])
def test_xcd_rank_is_an_xcd_major_bijection(lo):
    for hi in list(range(lo + 1, lo + 40)) + [lo + 255, lo + 256, lo + 511]:
        ranks = [xcd_rank(b, lo, hi) for b in range(lo, hi)]
        assert sorted(ranks) == list(range(hi - lo))
        by_rank = sorted(range(lo, hi), key=lambda b: xcd_rank(b, lo, hi))
        assert by_rank == sorted(range(lo, hi), key=lambda b: (b % K_XCDS, b))
