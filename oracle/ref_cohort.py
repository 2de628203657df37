"""ref_cohort — the reference's PK/PD cohorts, bit-faithful (JAX threefry draws restated).

TEST INFRASTRUCTURE ONLY (oracle/): imported by ``tests/`` and ``tests/golden/make_golden.py``.

``insite_ref.make_collection`` draws cohorts with numpy PCG64 (same distributions, different
numbers).  This module draws them exactly as the reference does, through ``oracle/jax_prng.py``:

* ``SyntheticPkpdDatasetCollection`` (``libs_m/ct/src/data/pkpd/dataset.py:557-607``): four
  subsets (train_f, val_f, test_cf_one_step, test_cf_treatment_seq), each constructed with the
  SAME ``seed`` (``:594-603``);
* ``SyntheticPkpdDataset.__init__`` (``dataset.py:52-72``): ``key = PRNGKey(seed)``;
  ``key, subkey = split(key)`` -> ``generate_params(..., key=subkey)``; ``key, subkey =
  split(key)`` -> the subset's simulator;
* ``get_standard_params`` (``pkpd_simulation.py:96-203``), ``simulate_factual`` (``:205-309``),
  ``simulate_counterfactual_1_step`` (``:352-471``), ``simulate_counterfactuals_treatment_seq``
  (``:516-667``, sliding-treatment mode, ``:474-487``) with their split/draw order, the
  ``jnp.arange`` time grids and the Euler-5 ``odeint`` (``utils.py:68-94``) on those grids.

With ``seed = 1`` (the logged ``exp.seed``, ``results/2_main_table/final_with_insite.txt:126``)
and the logged sizes (train 1000, val 100, test 100, T = 60, coeff 2) this reproduces the
reference's EQ_4_A..D cohorts: the oracle's discovery on them returns the logged 16-digit
equations to ~1e-15 (tests/test_reference_cohort.py).  EQ_4_M (``jax.random.choice``) is not
restated (no logged anchor).
"""
from __future__ import annotations

import numpy as np

from . import insite_ref as R
from . import jax_prng as J

SCALE = 0.5


def draw_params(num_patients: int, equation: str, key) -> dict:
    """``generate_params`` -> ``get_standard_params`` (pkpd_simulation.py:76-203)."""
    n = int(num_patients)
    key, sk = J.split(key)
    c_0 = J.normal(sk, (n,)) * (0.1 * SCALE) + 1.0 * SCALE                 # :117-118
    key, sk = J.split(key)
    c_1 = J.normal(sk, (n,)) * (0.1 * SCALE) + 1.0 * SCALE                 # :121-122
    C_0, C_1 = c_0, c_1                                                    # :126-127
    if equation in ("EQ_4_C", "EQ_4_D"):                                   # :128-150
        C_0 = 1.0 * c_0 + 0.1 * SCALE
        C_1 = 1.0 * c_1 + 0.3 * SCALE
        if equation == "EQ_4_D":                                           # :152-158
            key, sk = J.split(key)
            C_0 = J.normal(sk) * (0.5 * SCALE) + C_0
            key, sk = J.split(key)
            C_1 = J.normal(sk) * (0.5 * SCALE) + C_1
    elif equation not in ("EQ_4_A", "EQ_4_B"):
        raise NotImplementedError(f"{equation}: no threefry restatement (jax.random.choice)")
    C_0 = C_0 / 1.0                                                        # :178-179 (v = 1)
    C_1 = C_1 / 1.0
    key, sk = J.split(key)
    x0 = J.uniform(sk, (n,), 1.0, R.MAX_VALUE)                             # :181-182
    key, sk = J.split(key)
    idx = J.permutation(sk, np.arange(n))                                  # :195-197
    return {"initial_volumes": x0[idx], "hidden_C_0": np.asarray(C_0)[idx], "hidden_C_1": np.asarray(C_1)[idx],
            "observed_static_c_0": c_0[idx], "observed_static_c_1": c_1[idx]}


def _assign(x0, rv, conf_coeff):
    """``treatment_application_rv < sigmoid(gamma*(x0 - 25))`` (pkpd_simulation.py:88-89, 255-259)."""
    gamma = conf_coeff / R.MAX_VALUE
    prob = 1.0 / (1.0 + np.exp(-gamma * (x0 - R.MAX_VALUE / 2.0)))
    return (rv < prob).astype(np.int64)


def _odeint_interval(y, C, t0, t1):
    """``odeint(dy_dt, y, [t0, t1], ...)[1]`` (utils.py:86-90): HMAX < t1 - t0, so 5 Euler
    sub-steps of (t1 - t0)/5 with dy/dt = -C*y (pkpd_simulation.py:69-73)."""
    h = (t1 - t0) / R.STEPS_FOR_DT
    for _ in range(R.STEPS_FOR_DT):
        y = y + (-C * y) * h
    return y


def _noisy(equation):
    return equation.split("_")[-1] in ("B", "C", "D")


def simulate_factual(p, seq_length, key, equation, conf_coeff):
    """pkpd_simulation.py:205-309 (factual train/val cohorts)."""
    T = int(seq_length)
    dt = R.MAX_TIME_HORIZON / T
    x0 = p["initial_volumes"]
    n = x0.size
    key, sk = J.split(key)
    rec = J.uniform(sk, (n, T), 0.0, 1.0)                                  # :233-234
    key, sk = J.split(key)
    trv = J.uniform(sk, (n,), 0.0, 1.0)                                    # :235-236
    a = _assign(x0, trv, conf_coeff)
    C = np.where(a == 0, p["hidden_C_0"], p["hidden_C_1"])
    t = np.arange(0, R.MAX_TIME_HORIZON, dt)                               # :261
    V = np.empty((n, T))
    V[:, 0] = x0
    y = x0.copy()
    for k in range(T - 1):                                                 # :262 odeint over t
        y = _odeint_interval(y, C, t[k], t[k + 1])
        V[:, k + 1] = y
    seq = np.full(n, T - 1, dtype=np.int64)                                # :254
    recov = rec < np.exp(-V * R.RECOVERY_MULTIPLIER)                       # :264-265
    for i in np.nonzero(recov.any(axis=1))[0]:
        first = int(np.argmax(recov[i]))
        V[i] = V[i] * (np.arange(T) < first)
        seq[i] = first + 1
    dead = V > R.MAX_VALUE                                                 # :267-268
    for i in np.nonzero(dead.any(axis=1))[0]:
        first = int(np.argmax(dead[i]))
        m = np.arange(T) >= first
        V[i] = V[i] * (1 - m) + m * R.MAX_VALUE
        seq[i] = first + 1
    if _noisy(equation):                                                   # :289-291
        key, sk = J.split(key)
        V = V + R.OBSERVATION_NOISE * J.normal(sk, V.shape)
    treat = np.concatenate([np.repeat(a[:, None], T - 1, axis=1).astype(np.float64), np.zeros((n, 1))], axis=1)
    return {"cancer_volume": V, "treatment_application": treat, "sequence_lengths": seq.astype(np.float64),
            "observed_static_c_0": p["observed_static_c_0"].copy(), "observed_static_c_1": p["observed_static_c_1"].copy(),
            "hidden_C_0": p["hidden_C_0"].copy(), "hidden_C_1": p["hidden_C_1"].copy()}


def simulate_counterfactual_1_step(p, seq_length, key, equation, conf_coeff):
    """pkpd_simulation.py:352-471: per patient and step i, the factual row V[0..i+1] and the
    counterfactual row V[0..i] + one Euler-5 interval under 1 - a; N*(T-1)*2 rows."""
    T = int(seq_length)
    dt = R.MAX_TIME_HORIZON / T
    x0 = p["initial_volumes"]
    n = x0.size
    key, sk = J.split(key)
    J.uniform(sk, (n, T - 1), 0.0, 1.0)                                    # :380-381 recovery rvs (unused)
    key, sk = J.split(key)
    trv = J.uniform(sk, (n,), 0.0, 1.0)                                    # :382-383
    a = _assign(x0, trv, conf_coeff)
    C = np.where(a == 0, p["hidden_C_0"], p["hidden_C_1"])
    Ccf = np.where(a == 0, p["hidden_C_1"], p["hidden_C_0"])
    t = np.arange(0, R.MAX_TIME_HORIZON, dt)                               # :394-395
    V = np.empty((n, T))
    V[:, 0] = x0
    cf = np.empty((n, T - 1))
    for k in range(T - 1):                                                 # scan :341-350, 397
        cf[:, k] = _odeint_interval(V[:, k], Ccf, t[k], t[k + 1])
        V[:, k + 1] = _odeint_interval(V[:, k], C, t[k], t[k + 1])
    reps = (T - 1) * 2
    vol = np.zeros((n, reps, T))
    trt = np.zeros((n, reps, T - 1))
    sl = np.zeros((n, reps), dtype=np.int64)
    for i in range(T - 1):                                                 # :406-415
        vol[:, 2 * i, :i + 2] = V[:, :i + 2]
        trt[:, 2 * i, :i + 1] = a[:, None]
        sl[:, 2 * i] = i + 1
        vol[:, 2 * i + 1, :i + 1] = V[:, :i + 1]
        vol[:, 2 * i + 1, i + 1] = cf[:, i]
        trt[:, 2 * i + 1, :i] = a[:, None]
        trt[:, 2 * i + 1, i] = 1 - a
        sl[:, 2 * i + 1] = i + 1
    if _noisy(equation):                                                   # :442-444
        key, sk = J.split(key)
        vol = vol + R.OBSERVATION_NOISE * J.normal(sk, vol.shape)
    rows = n * reps
    return {"cancer_volume": vol.reshape(rows, T),
            "treatment_application": np.concatenate([trt.reshape(rows, T - 1), np.zeros((rows, 1))], axis=1),
            "sequence_lengths": sl.reshape(rows).astype(np.float64),
            "observed_static_c_0": np.repeat(p["observed_static_c_0"], reps),
            "observed_static_c_1": np.repeat(p["observed_static_c_1"], reps)}


def simulate_counterfactuals_treatment_seq(p, seq_length, projection_horizon, key, equation, conf_coeff):
    """pkpd_simulation.py:516-667 (sliding_treatment, :474-487): per step i the factual state
    V[i+1] is rolled tau intervals under 2*tau plans (eye / 1 - eye); N*(T-1)*2*tau rows."""
    T = int(seq_length)
    tau = int(projection_horizon)
    dt = R.MAX_TIME_HORIZON / T
    t = np.arange(0, T + 1).astype(np.float64) * dt                        # :537
    x0 = p["initial_volumes"]
    n = x0.size
    key, sk = J.split(key)
    J.uniform(sk, (n, T + tau - 1), 0.0, 1.0)                              # :555-556 recovery rvs (unused)
    key, sk = J.split(key)
    trv = J.uniform(sk, (n,), 0.0, 1.0)                                    # :557-558
    a = _assign(x0, trv, conf_coeff)
    C0, C1 = p["hidden_C_0"], p["hidden_C_1"]
    C = np.where(a == 0, C0, C1)
    plans = np.concatenate([np.eye(tau, dtype=np.int64), 1 - np.eye(tau, dtype=np.int64)], axis=0)   # :476
    V = np.empty((n, T + 1))
    V[:, 0] = x0
    V[:, 1] = _odeint_interval(x0, C, t[0], t[1])                          # :574
    cfv = np.empty((n, T - 1, 2 * tau, tau))
    for i in range(T - 1):                                                 # t_tuples (t[i+1], t[i+2]) :571
        t_s, t_e = t[i + 1], t[i + 2]
        vcur = V[:, i + 1]
        for q in range(2 * tau):                                           # :478-486
            v = vcur
            cs, ce = t_s, t_e
            for j in range(tau):
                v = _odeint_interval(v, np.where(plans[q, j] == 0, C0, C1), cs, ce)
                cs, ce = cs + dt, ce + dt
                cfv[:, i, q, j] = v
        V[:, i + 2] = _odeint_interval(vcur, C, t_s, t_e)                  # :513
    L = T + tau
    nr = (T - 1) * 2 * tau
    vol = np.zeros((n, nr, L))
    trt = np.zeros((n, nr, L - 1))
    sl = np.zeros((n, nr), dtype=np.int64)
    r = 0
    for i in range(T - 1):                                                 # :593-597
        for q in range(2 * tau):
            vol[:, r, :i + 2] = V[:, :i + 2]
            vol[:, r, i + 2:i + 2 + tau] = cfv[:, i, q, :]
            trt[:, r, :i + 1] = a[:, None]
            trt[:, r, i + 1:i + 1 + tau] = plans[q][None, :]
            sl[:, r] = i + 1 + tau
            r += 1
    key = J.split(key, n + 1)[0]                                           # :616 key, *subkeys = split(key, n+1)
    if _noisy(equation):                                                   # :639-641
        key, sk = J.split(key)
        vol = vol + R.OBSERVATION_NOISE * J.normal(sk, vol.shape)
    rows = n * nr
    return {"cancer_volume": vol.reshape(rows, L),
            "treatment_application": np.concatenate([trt.reshape(rows, L - 1), np.zeros((rows, 1))], axis=1),
            "sequence_lengths": sl.reshape(rows).astype(np.float64),
            "observed_static_c_0": np.repeat(p["observed_static_c_0"], nr),
            "observed_static_c_1": np.repeat(p["observed_static_c_1"], nr)}


def _subset_keys(seed):
    """dataset.py:52-54, 64/67/71: params subkey, then simulator subkey."""
    key = J.PRNGKey(seed)
    key, k_params = J.split(key)
    key, k_sim = J.split(key)
    return k_params, k_sim


def make_collection(equation="EQ_4_A", num_patients=None, seq_length=60, projection_horizon=5, conf_coeff=2,
                    seed=1, with_tests=True, treatment_mode="multiclass"):
    """``SyntheticPkpdDatasetCollection`` + ``process_data_multi`` with the reference's draws.
    Returns the same {name: insite_ref.Subset} mapping as ``insite_ref.make_collection``."""
    num_patients = num_patients or {"train": 1000, "val": 100, "test": 100}
    sims = {}
    for name in ("train", "val"):                                          # dataset.py:594-595
        kp, ks = _subset_keys(seed)
        p = draw_params(num_patients[name], equation, kp)
        sims[name] = simulate_factual(p, seq_length, ks, equation, conf_coeff)
    if with_tests:
        kp, ks = _subset_keys(seed)                                        # :596-598
        p = draw_params(num_patients["test"], equation, kp)
        sims["test_cf_one_step"] = simulate_counterfactual_1_step(p, seq_length, ks, equation, conf_coeff)
        kp, ks = _subset_keys(seed)                                        # :599-603
        p = draw_params(num_patients["test"], equation, kp)
        sims["test_cf_treatment_seq"] = simulate_counterfactuals_treatment_seq(p, seq_length, projection_horizon, ks,
                                                                              equation, conf_coeff)
    scaling = R.get_scaling_params(sims["train"])                          # dataset.py:607
    out = {}
    for name, sim in sims.items():                                         # process_data_multi
        d, sp = R.process_data(sim, scaling, treatment_mode)
        out[name] = R.Subset(name, d, sp)
    if with_tests:
        s = out["test_cf_treatment_seq"]
        s.data_processed_seq = R.process_sequential_test(s.data, s.scaling_params, projection_horizon)
    return out
