"""The on-device cohort generator (csrc/insite_rng.hip + insite_amd/threefry.py + insite_amd/pkpd.py
rng="threefry") against the Threefry known answers, the numpy restatement of jax.random
(oracle/jax_prng.py) and the reference's own cohorts (oracle/ref_cohort.py), and end to end: ``run.py``
on the device-drawn cohorts reproduces the published EQ_4 run rows
(results/2_main_table/final_with_insite.txt:126,154,182,210; tests/golden/reference_log_anchors.json).

Tolerances: words, uniforms and permutations bit-exact (integer work); normals rtol 1e-12 (torch's
float64 erfinv vs scipy's, a few ulp); cohort arrays 1e-12 absolute on O(1) normalised values;
discovered equations 1e-10 L-inf with identical support and RMSE metrics 1e-9 relative (the bar of
tests/test_gpu_reference.py, where the cohorts come from the CPU oracle instead).
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import jax_prng as J
from oracle import ref_cohort as RC

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ANCHORS = json.load(open(os.path.join(HERE, "golden", "reference_log_anchors.json")))


def _tf():
    from insite_amd import threefry
    return threefry


@pytest.mark.parametrize("key,ctr,out", [
    ((0x00000000, 0x00000000), (0x00000000, 0x00000000), (0x6B200159, 0x99BA4EFE)),
    ((0xFFFFFFFF, 0xFFFFFFFF), (0xFFFFFFFF, 0xFFFFFFFF), (0x1CB996FC, 0xBB002BE7)),
    ((0x13198A2E, 0x03707344), (0x243F6A88, 0x85A308D3), (0xC4923A9C, 0x483DF7A0)),
])
def test_random123_kat_through_iota_layout(dev, key, ctr, out):
    """The kernel hashes (j, j + n/2): with n = 2 and key k, thread 0 hashes (0, 1).  The KAT counters
    are reached by the oracle block function, which the iota words then must match pairwise."""
    tf = _tf()
    if ctr == (0, 0):
        w = tf._words(key, 1, dev).cpu().tolist()      # odd count: (0, pad 0) -> word 0 of the block
        assert w == [out[0]]
    a, b = J.threefry2x32_block(key[0], key[1], np.array([ctr[0]], np.uint32), np.array([ctr[1]], np.uint32))
    assert (int(a[0]), int(b[0])) == out
    w2 = tf._words(key, 2, dev).cpu().numpy()
    y0, y1 = J.threefry2x32_block(key[0], key[1], np.array([0], np.uint32), np.array([1], np.uint32))
    assert w2.tolist() == [int(y0[0]), int(y1[0])]


@pytest.mark.parametrize("n", [1, 2, 3, 64, 255, 1001, (1 << 20) + 7])
def test_iota_words_match_oracle(dev, n):
    tf = _tf()
    for key in ((0, 0), (0, 1), (0x9E3779B9, 0x7F4A7C15)):
        got = tf._words(key, n, dev).cpu().numpy().astype(np.uint32)
        ref = J.threefry_2x32(np.array(key, np.uint32), np.arange(n, dtype=np.uint32))
        assert np.array_equal(got, ref), (key, n)


def test_split_documented_value(dev):
    tf = _tf()
    assert tf.prng_key(0) == (0, 0)
    assert tf.split((0, 0), 2, dev) == [(4146024105, 967050713), (2718843009, 1272950319)]
    k = tf.prng_key(123)
    assert [list(p) for p in tf.split(k, 5, dev)] == J.split(J.PRNGKey(123), 5).tolist()


def test_transforms_match_oracle(dev):
    tf = _tf()
    k = (0, 42)
    kj = np.array(k, np.uint32)
    for shape in [(), (1,), (7,), (33, 17)]:
        u = tf.uniform(k, shape, dev, 1.0, 50.0).cpu().numpy()
        assert np.array_equal(u, J.uniform(kj, shape, 1.0, 50.0)), shape
        b = tf.random_bits(k, 64, shape, dev).cpu().numpy().astype(np.uint64)
        assert np.array_equal(b, J.random_bits(kj, 64, shape)), shape
    z = tf.normal(k, (200_000,), dev).cpu().numpy()
    zr = J.normal(kj, (200_000,))
    np.testing.assert_allclose(z, zr, rtol=1e-12, atol=1e-15)
    for n in (1, 2, 100, 1000, 5000):
        p = tf.permutation(k, n, dev).cpu().numpy()
        assert np.array_equal(p, J.permutation(kj, np.arange(n))), n


def test_stream_key_threading_matches_reference_pattern(dev):
    """``key, subkey = split(key)`` before every draw; ``split_first`` = ``key = split(key, n)[0]``."""
    tf = _tf()
    s = tf.Stream(tf.prng_key(9), dev)
    key = J.PRNGKey(9)
    for _ in range(3):
        got = s.normal(5).cpu().numpy()
        key, sk = J.split(key)
        np.testing.assert_allclose(got, J.normal(sk, (5,)), rtol=1e-12, atol=1e-15)
    s.split_first(11)
    key = J.split(key, 11)[0]
    assert s.key == (int(key[0]), int(key[1]))


def _dev_collection(eq, dev, seed=1):
    from insite_amd import pkpd
    return pkpd.dataset_collection(eq, {"train": 1000, "val": 100, "test": 100}, seed=seed, device=dev,
                                   rng="threefry")


@pytest.mark.parametrize("eq", ["EQ_4_A", "EQ_4_D"])
def test_device_cohort_matches_reference_cohort(dev, eq):
    """pkpd.py with rng='threefry' draws the reference's cohorts: every processed array of every subset."""
    c = _dev_collection(eq, dev)
    ref = RC.make_collection(eq)
    subsets = {"train": c.train_f, "val": c.val_f, "test_cf_one_step": c.test_cf_one_step,
               "test_cf_treatment_seq": c.test_cf_treatment_seq}
    for name, ds in subsets.items():
        r = ref[name].data
        for k in ("sequence_lengths", "current_treatments", "active_entries"):
            assert np.array_equal(np.asarray(ds.data[k]), np.asarray(r[k])), (name, k)
        for k in ("prev_outputs", "outputs", "static_features", "unscaled_outputs"):
            np.testing.assert_allclose(ds.data[k], r[k], rtol=0, atol=1e-11, err_msg=f"{name}/{k}")
    sq, rq = c.test_cf_treatment_seq.data_processed_seq, ref["test_cf_treatment_seq"].data_processed_seq
    np.testing.assert_allclose(sq["outputs"], rq["outputs"], rtol=0, atol=1e-11)


def test_eq4m_choice_draws_both_modes(dev):
    """EQ_4_M (jax.random.choice over {0.1, 0.3} x 0.5; no logged anchor, parity unpinned): both modes
    drawn about equally, each patient's C - c one of the two means."""
    from insite_amd import pkpd
    rp, _ = pkpd.subset_rngs("threefry", 3, "train", dev)
    p = pkpd.draw_params(4000, "EQ_4_M", rp)
    d = (p["hidden_C_0"] - p["observed_static_c_0"]).cpu().numpy()
    hi = np.isclose(d, 0.15, atol=1e-12)
    lo = np.isclose(d, 0.05, atol=1e-12)
    assert np.all(hi | lo) and 0.45 < hi.mean() < 0.55


@pytest.mark.parametrize("eq", ["EQ_4_A", "EQ_4_B", "EQ_4_C", "EQ_4_D"])
def test_run_py_reproduces_logged_rows(dev, eq):
    """``run.py``'s run list entry (dataset, 'sindy', seed 1) with every draw made on the device."""
    import run
    from insite_amd import config as C
    from test_gpu_reference import METRICS, logged_coefs
    driver = C.driver_config()
    driver["setup"]["debug_mode"] = True
    r = run.run_one(driver, eq, "sindy", 1, driver["run"]["domain_conf"], device=dev)
    anchor = ANCHORS[f"{eq}/sindy"]
    got = logged_coefs(r["global_equation_string"])
    ref = logged_coefs(anchor["global_equation_string"])
    assert np.array_equal(got != 0, ref != 0)
    assert np.max(np.abs(got - ref)) < 1e-10
    for k in METRICS:
        assert r[k] == pytest.approx(anchor[k], rel=1e-9), k
    assert r["seed"] == 1 and r["errored"] is False
