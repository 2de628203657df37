"""insite_ref — CPU restatement (numpy, fp64) of the INSITE ODE-discovery hot path.

TEST INFRASTRUCTURE ONLY.  This module is the parity oracle: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it, and there only as the checker / the timed CPU baseline.  The product path
(``insite_amd``) never imports, links or calls anything under ``oracle/``.

Parity status
-------------
The reference (samholt/ODE-Discovery-for-Longitudinal-Heterogeneous-Treatment-
Effects-Inference, "INSITE") is Python/JAX and cannot be imported here: jax,
pysindy, sympy2jax, hydra, omegaconf, lightning are absent (ordinary
ModuleNotFoundError, no permission denial).  The SINDy arithmetic
lives in third-party **pysindy** (not vendored, version unpinned:
``setup/requirements.txt:1``; the 1.7.x API is inferred from the call sites
``libs_m/ct/src/models/sindy.py:186-271``).  This module therefore restates:

* the reference's own code paths, cited file:line below (integrator, STLSQ
  semantics copied in-repo as ``LSQIntialMask``, RHS construction, DE-format
  extraction, cohort generator, dataset layout, metrics);
* pysindy 1.7.x's published algorithm for SmoothedFiniteDifference (scipy
  ``savgol_filter(window 5, polyorder 3, mode='interp')`` then the 4th-order
  5-point finite difference with one-sided 5-point end stencils),
  PolynomialLibrary column order, STLSQ (all-ones initial support, ridge via
  sklearn's Cholesky solver, thresholding, stop rule) and the post-fit unbias
  (unregularised least squares on the support).

It is pinned against REFERENCE-HELD OUTPUTS: ``oracle/ref_cohort.py`` regenerates the
reference's own EQ_4_A..D cohorts bit for bit (jax threefry restated in ``oracle/jax_prng.py``,
seed 1 as logged), and this module's discovery on them returns the 16-digit equations of
``results/2_main_table/final_with_insite.txt:126,154,182,210`` to ~1e-15, and its rollout +
metrics the logged RMSEs (tests/test_reference_cohort.py).  That pins the savgol(5,3) stencils,
pysindy's one-sided 5-point FD4 end stencils, the library on the RAW x (smoothing feeds x_dot
only), STLSQ + unbias, the Euler-5 rollout and the metric definitions.  Further pins
(tests/test_oracle.py): the sub-oracles the reference's dependencies delegate to
(``scipy.signal.savgol_filter``, ``sklearn.linear_model.ridge_regression``,
``numpy.linalg.lstsq``, ``scipy.integrate.solve_ivp``) and the reference's in-module
known-answer test for the integrator (``libs_m/ct/src/data/pkpd/utils.py:759-858``).

``make_collection`` below draws cohorts with numpy PCG64 (same distributions, fast, any size);
``ref_cohort.make_collection`` is the bit-faithful variant.  The PCG64 path uses the time grid
``k*dt`` with a constant Euler sub-step ``dt/5`` (the reference's ``arange`` grid differs by ulps)
and passes ``dt`` consistently to model and generator (reference hard-codes ``STANDARD_DT``;
SURVEY.md F9).
"""
from __future__ import annotations

import itertools
import math
from dataclasses import dataclass, field

import numpy as np

# --------------------------------------------------------------------------------------
# Constants — libs_m/ct/src/data/pkpd/utils.py:37-54
# --------------------------------------------------------------------------------------
MAX_VALUE = 50.0                      # utils.py:37
STEPS_FOR_DT = 5                      # utils.py:40
MAX_TIME_HORIZON = 10.0               # utils.py:48
MAX_SEQUENCE_LENGTH = 60              # utils.py:51
STANDARD_DT = MAX_TIME_HORIZON / MAX_SEQUENCE_LENGTH   # utils.py:53
HMAX = STANDARD_DT / STEPS_FOR_DT     # utils.py:54
OBSERVATION_NOISE = 0.01              # pkpd_simulation.py:44
RECOVERY_MULTIPLIER = 5.8 * 10 ** (8 + 3)   # pkpd_simulation.py:46
RHS_COEF_EPS = 1e-3                   # utils.py:388  (|coef| > 1e-3 kept in the RHS)
SUPPORT_EPS = 1e-14                   # pysindy BaseOptimizer: ind_ = |coef| > 1e-14

EQUATIONS = ("EQ_4_A", "EQ_4_B", "EQ_4_C", "EQ_4_D", "EQ_4_M")


# --------------------------------------------------------------------------------------
# A11 — cohort generator (pkpd_simulation.py:76-203, 205-309, 341-471, 474-667)
# --------------------------------------------------------------------------------------
def draw_params(num_patients: int, equation: str, rng: np.random.Generator) -> dict:
    """Patient parameters; distributions of ``get_standard_params`` (pkpd_simulation.py:96-203).

    Draw order (our RNG protocol, PCG64): c_0, c_1, [EQ_4_D: C_0 shift, C_1 shift]
    [EQ_4_M: means_0, means_1], initial volumes, permutation.
    """
    scale = 0.5
    n = int(num_patients)
    c_0 = rng.standard_normal(n) * (0.1 * scale) + 1.0 * scale      # :117-118
    c_1 = rng.standard_normal(n) * (0.1 * scale) + 1.0 * scale      # :121-122
    C_0, C_1 = c_0.copy(), c_1.copy()                               # :125-127 (EQ_4_A/B)
    if equation in ("EQ_4_C", "EQ_4_D"):                            # :128-150
        C_0 = 1.0 * c_0 + 0.1 * scale
        C_1 = 1.0 * c_1 + 0.3 * scale
        if equation == "EQ_4_D":                                    # :152-158 one scalar per arm
            C_0 = rng.standard_normal() * (0.5 * scale) + C_0
            C_1 = rng.standard_normal() * (0.5 * scale) + C_1
    elif equation == "EQ_4_M":                                      # :159-165
        C_0 = c_0 + rng.choice(np.array([0.1, 0.3]) * scale, size=n)
        C_1 = c_1 + rng.choice(np.array([0.1, 0.3]) * scale, size=n)
    elif equation not in ("EQ_4_A", "EQ_4_B"):
        raise NotImplementedError(equation)
    x0 = rng.uniform(1.0, MAX_VALUE, size=n)                        # :182
    idx = rng.permutation(n)                                        # :196-201
    return {
        "initial_volumes": x0[idx],
        "hidden_C_0": np.asarray(C_0, dtype=np.float64)[idx],
        "hidden_C_1": np.asarray(C_1, dtype=np.float64)[idx],
        "observed_static_c_0": c_0[idx],
        "observed_static_c_1": c_1[idx],
    }


def _treatment_assignment(x0, rv, conf_coeff):
    """Bernoulli(sigmoid(gamma/50*(x0-25))) (pkpd_simulation.py:76-94, 255-259)."""
    gamma = conf_coeff / MAX_VALUE
    prob = 1.0 / (1.0 + np.exp(-gamma * (x0 - MAX_VALUE / 2.0)))
    return (rv < prob).astype(np.int64)


def _euler5_decay(v, C, dt):
    """One observation interval of the true model dy/dt = -C*y (pkpd_simulation.py:69-74)
    with the reference integrator: 5 forward-Euler sub-steps of h = dt/5 (utils.py:68-79)."""
    h = dt / STEPS_FOR_DT
    for _ in range(STEPS_FOR_DT):
        v = v + (-C * v) * h
    return v


def _arm_rate(arm, C0, C1):
    return np.where(arm == 0, C0, C1)


def simulate_factual(params, seq_length, rng, equation, conf_coeff):
    """Factual cohort (pkpd_simulation.py:205-309). Returns the reference's data dict."""
    T = int(seq_length)
    dt = MAX_TIME_HORIZON / T
    x0 = params["initial_volumes"]
    n = x0.shape[0]
    recovery_rvs = rng.uniform(0.0, 1.0, size=(n, T))              # :250
    treat_rvs = rng.uniform(0.0, 1.0, size=n)                      # :252
    a = _treatment_assignment(x0, treat_rvs, conf_coeff)
    C = _arm_rate(a, params["hidden_C_0"], params["hidden_C_1"])
    V = np.empty((n, T))
    V[:, 0] = x0
    for k in range(1, T):                                          # :262 odeint over t grid
        V[:, k] = _euler5_decay(V[:, k - 1], C, dt)
    seq = np.full(n, T - 1, dtype=np.int64)                        # :254
    # recovery (:264-265) / death (:267-268) masks, applied per patient
    rec = recovery_rvs < np.exp(-V * RECOVERY_MULTIPLIER)
    for i in np.nonzero(rec.any(axis=1))[0]:
        first = int(np.argmax(rec[i]))
        V[i] = V[i] * (np.arange(T) < first)
        seq[i] = first + 1
    dead = V > MAX_VALUE
    for i in np.nonzero(dead.any(axis=1))[0]:
        first = int(np.argmax(dead[i]))
        m = np.arange(T) >= first
        V[i] = V[i] * (1 - m) + m * MAX_VALUE
        seq[i] = first + 1
    if equation.split("_")[-1] in ("B", "C", "D"):                # :289-291
        V = V + OBSERVATION_NOISE * rng.standard_normal(V.shape)
    treat = np.concatenate([np.repeat(a[:, None], T - 1, axis=1).astype(np.float64),
                            np.zeros((n, 1))], axis=1)              # :270,296
    return {
        "cancer_volume": V,
        "treatment_application": treat,
        "sequence_lengths": seq.astype(np.float64),
        "observed_static_c_0": params["observed_static_c_0"].copy(),
        "observed_static_c_1": params["observed_static_c_1"].copy(),
        # generator ground truth (not read by the model)
        "hidden_C_0": params["hidden_C_0"].copy(),
        "hidden_C_1": params["hidden_C_1"].copy(),
    }


def simulate_counterfactual_1_step(params, seq_length, rng, equation, conf_coeff):
    """All one-step-ahead counterfactuals (pkpd_simulation.py:341-471); N*(T-1)*2 rows."""
    T = int(seq_length)
    dt = MAX_TIME_HORIZON / T
    x0 = params["initial_volumes"]
    n = x0.shape[0]
    rng.uniform(0.0, 1.0, size=(n, T - 1))                          # recovery rvs (:375), unused
    treat_rvs = rng.uniform(0.0, 1.0, size=n)                       # :377
    a = _treatment_assignment(x0, treat_rvs, conf_coeff)
    C = _arm_rate(a, params["hidden_C_0"], params["hidden_C_1"])
    Ccf = _arm_rate(1 - a, params["hidden_C_0"], params["hidden_C_1"])
    V = np.empty((n, T))
    V[:, 0] = x0
    cf = np.empty((n, T - 1))
    for k in range(T - 1):                                          # scan :344-350
        cf[:, k] = _euler5_decay(V[:, k], Ccf, dt)
        V[:, k + 1] = _euler5_decay(V[:, k], C, dt)
    rows = n * (T - 1) * 2
    vol = np.zeros((n, (T - 1) * 2, T))
    trt = np.zeros((n, (T - 1) * 2, T - 1))
    sl = np.zeros((n, (T - 1) * 2), dtype=np.int64)
    for i in range(T - 1):                                          # :405-413
        vol[:, 2 * i, :i + 2] = V[:, :i + 2]
        trt[:, 2 * i, :i + 1] = a[:, None]
        sl[:, 2 * i] = i + 1
        vol[:, 2 * i + 1, :i + 1] = V[:, :i + 1]
        vol[:, 2 * i + 1, i + 1] = cf[:, i]
        trt[:, 2 * i + 1, :i] = a[:, None]
        trt[:, 2 * i + 1, i] = 1 - a
        sl[:, 2 * i + 1] = i + 1
    if equation.split("_")[-1] in ("B", "C", "D"):                 # :438-440
        vol = vol + OBSERVATION_NOISE * rng.standard_normal(vol.shape)
    reps = (T - 1) * 2
    return {
        "cancer_volume": vol.reshape(rows, T),
        "treatment_application": np.concatenate([trt.reshape(rows, T - 1), np.zeros((rows, 1))], axis=1),
        "sequence_lengths": sl.reshape(rows).astype(np.float64),
        "observed_static_c_0": np.repeat(params["observed_static_c_0"], reps),
        "observed_static_c_1": np.repeat(params["observed_static_c_1"], reps),
    }


def simulate_counterfactuals_treatment_seq(params, seq_length, projection_horizon, rng, equation, conf_coeff):
    """tau-step sliding-treatment counterfactuals (pkpd_simulation.py:474-487, 516-667);
    N*(T-1)*2*tau rows of length T+tau."""
    T = int(seq_length)
    tau = int(projection_horizon)
    dt = MAX_TIME_HORIZON / T
    x0 = params["initial_volumes"]
    n = x0.shape[0]
    rng.uniform(0.0, 1.0, size=(n, T + tau - 1))                    # recovery rvs (:571), unused
    treat_rvs = rng.uniform(0.0, 1.0, size=n)                       # :573
    a = _treatment_assignment(x0, treat_rvs, conf_coeff)
    C0, C1 = params["hidden_C_0"], params["hidden_C_1"]
    C = _arm_rate(a, C0, C1)
    plans = np.concatenate([np.eye(tau, dtype=np.int64), 1 - np.eye(tau, dtype=np.int64)], axis=0)  # :489
    V = np.empty((n, T + 1))
    V[:, 0] = x0
    V[:, 1] = _euler5_decay(x0, C, dt)                               # :593
    cfv = np.empty((n, T - 1, 2 * tau, tau))
    for i in range(T - 1):                                           # scan over t_tuples :600
        vcur = V[:, i + 1]
        for p in range(2 * tau):
            v = vcur
            for j in range(tau):
                v = _euler5_decay(v, _arm_rate(np.full(n, plans[p, j]), C0, C1), dt)
                cfv[:, i, p, j] = v
        V[:, i + 2] = _euler5_decay(vcur, C, dt)
    L = T + tau
    nr = (T - 1) * 2 * tau
    vol = np.zeros((n, nr, L))
    trt = np.zeros((n, nr, L - 1))
    sl = np.zeros((n, nr), dtype=np.int64)
    r = 0
    for i in range(T - 1):                                           # :608-613
        for p in range(2 * tau):
            vol[:, r, :i + 2] = V[:, :i + 2]
            vol[:, r, i + 2:i + 2 + tau] = cfv[:, i, p, :]
            trt[:, r, :i + 1] = a[:, None]
            trt[:, r, i + 1:i + 1 + tau] = plans[p][None, :]
            sl[:, r] = i + 1 + tau
            r += 1
    if equation.split("_")[-1] in ("B", "C", "D"):                  # :644-646
        vol = vol + OBSERVATION_NOISE * rng.standard_normal(vol.shape)
    rows = n * nr
    return {
        "cancer_volume": vol.reshape(rows, L),
        "treatment_application": np.concatenate([trt.reshape(rows, L - 1), np.zeros((rows, 1))], axis=1),
        "sequence_lengths": sl.reshape(rows).astype(np.float64),
        "observed_static_c_0": np.repeat(params["observed_static_c_0"], nr),
        "observed_static_c_1": np.repeat(params["observed_static_c_1"], nr),
    }


def get_scaling_params(sim):
    """Mean/std over active entries (pkpd_simulation.py:670-693)."""
    seq = sim["sequence_lengths"].astype(np.int64)
    vals = np.concatenate([sim["cancer_volume"][i, :seq[i]] for i in range(seq.shape[0])])
    means = {"cancer_volume": float(np.mean(vals)),
             "observed_static_c_0": float(np.mean(sim["observed_static_c_0"])),
             "observed_static_c_1": float(np.mean(sim["observed_static_c_1"]))}
    stds = {"cancer_volume": float(np.std(vals)),
            "observed_static_c_0": float(np.std(sim["observed_static_c_0"])),
            "observed_static_c_1": float(np.std(sim["observed_static_c_1"]))}
    return means, stds


def process_data(sim, scaling, treatment_mode="multiclass"):
    """Layout of ``SyntheticPkpdDataset.process_data`` (pkpd/dataset.py:96-192): multiclass one-hot
    treatments [N, T-1, 2] (:135-147) or multilabel [N, T-1, 1] (:149-151, the joint-model ablation's
    ``dataset.treatment_mode=multilabel``, run.py:198-201)."""
    mean, std = scaling
    d = dict(sim)
    V = (sim["cancer_volume"] - mean["cancer_volume"]) / std["cancer_volume"]
    c0 = (sim["observed_static_c_0"] - mean["observed_static_c_0"]) / std["observed_static_c_0"]
    c1 = (sim["observed_static_c_1"] - mean["observed_static_c_1"]) / std["observed_static_c_1"]
    app = sim["treatment_application"][:, :-1]                       # :132-133
    if treatment_mode == "multiclass":
        onehot = np.zeros(app.shape + (2,))
        onehot[..., 0] = (app == 0)
        onehot[..., 1] = (app == 1)
    elif treatment_mode == "multilabel":
        onehot = app[..., None].astype(np.float64)
    else:
        raise ValueError(treatment_mode)
    seq = sim["sequence_lengths"]
    Tm1 = V.shape[1] - 1
    cur_cov = np.stack([V[:, :-1], np.repeat(c0[:, None], Tm1, 1), np.repeat(c1[:, None], Tm1, 1)], axis=-1)
    outputs = V[:, 1:, None]
    active = np.zeros(outputs.shape)
    for i in range(seq.shape[0]):
        active[i, :int(seq[i]), :] = 1
    d["current_treatments"] = onehot
    d["prev_treatments"] = np.concatenate([np.zeros((V.shape[0], 1, onehot.shape[-1])), onehot[:, :-1, :]], axis=1)
    d["current_covariates"] = cur_cov
    d["outputs"] = outputs
    d["active_entries"] = active
    d["unscaled_outputs"] = outputs * std["cancer_volume"] + mean["cancer_volume"]
    d["prev_outputs"] = cur_cov[:, :, :1]
    d["static_features"] = cur_cov[:, 0, 1:]
    scaling_params = {
        "input_means": np.array([mean["cancer_volume"], mean["observed_static_c_0"], mean["observed_static_c_1"], 0.0]),
        "inputs_stds": np.array([std["cancer_volume"], std["observed_static_c_0"], std["observed_static_c_1"], 1.0]),
        "output_means": mean["cancer_volume"],
        "output_stds": std["cancer_volume"],
    }
    return d, scaling_params


def process_sequential_test(data, scaling_params, projection_horizon):
    """``process_sequential_test`` targets (pkpd/dataset.py:395-475): the last tau outputs per row."""
    tau = int(projection_horizon)
    seq = data["sequence_lengths"].astype(np.int64)
    n = seq.shape[0]
    out = np.zeros((n, tau, 1))
    for i in range(n):
        fl = int(seq[i]) - tau
        out[i] = data["outputs"][i, fl:fl + tau, :]
    return {"outputs": out, "active_entries": np.ones((n, tau, 1)),
            "unscaled_outputs": out * scaling_params["output_stds"] + scaling_params["output_means"]}


@dataclass
class Subset:
    name: str
    data: dict
    scaling_params: dict
    data_processed_seq: dict | None = None
    norm_const: float = MAX_VALUE


def make_collection(equation="EQ_4_A", num_patients=None, seq_length=60, projection_horizon=5,
                    conf_coeff=2.0, seed=0, with_tests=True, treatment_mode="multiclass"):
    """``SyntheticPkpdDatasetCollection`` + ``process_data_multi`` (pkpd/dataset.py:557-607;
    dataset_collection.py:74-86).  Subsets use independent child streams of ``seed``."""
    num_patients = num_patients or {"train": 500, "val": 100, "test": 100}
    ss = np.random.SeedSequence(seed)
    kids = ss.spawn(4)
    out = {}
    sims = {}
    for kid, name in zip(kids[:2], ("train", "val")):
        rng = np.random.default_rng(kid)
        p = draw_params(num_patients[name], equation, rng)
        sims[name] = simulate_factual(p, seq_length, rng, equation, conf_coeff)
    if with_tests:
        rng = np.random.default_rng(kids[2])
        p = draw_params(num_patients["test"], equation, rng)
        sims["test_cf_one_step"] = simulate_counterfactual_1_step(p, seq_length, rng, equation, conf_coeff)
        rng = np.random.default_rng(kids[3])
        p = draw_params(num_patients["test"], equation, rng)
        sims["test_cf_treatment_seq"] = simulate_counterfactuals_treatment_seq(
            p, seq_length, projection_horizon, rng, equation, conf_coeff)
    scaling = get_scaling_params(sims["train"])
    for name, sim in sims.items():
        d, sp = process_data(sim, scaling, treatment_mode)
        out[name] = Subset(name, d, sp)
    if with_tests:
        s = out["test_cf_treatment_seq"]
        s.data_processed_seq = process_sequential_test(s.data, s.scaling_params, projection_horizon)
    return out


# --------------------------------------------------------------------------------------
# A1 — DE-format extraction (pkpd/utils.py:419-432, 523-606), EQ_4 non-joint
# --------------------------------------------------------------------------------------
def unscale_inputs(data, scaling_params, dim_outcome=1, dim_static=2):
    sp = scaling_params
    prev = data["prev_outputs"] * sp["output_stds"] + sp["output_means"]           # :543
    stat = (data["static_features"] * sp["inputs_stds"][dim_outcome:dim_outcome + dim_static]
            + sp["input_means"][dim_outcome:dim_outcome + dim_static])             # :545
    return prev[..., 0], stat


def de_format(data, scaling_params, sequence_lengths_offset=1):
    """Dense DE layout: reconstructed volume ``x[N,T]`` (utils.py:554), statics ``u[N,2]``,
    per-patient arm (``treatments[0]==[1,0]`` -> 0, utils.py:425) and row count
    ``seq_len - offset`` (utils.py:426)."""
    prev, stat = unscale_inputs(data, scaling_params)
    unscaled_outputs = data["unscaled_outputs"][..., 0]
    x = np.concatenate([prev[:, :1], unscaled_outputs], axis=1)
    ct = data["current_treatments"]
    arm = np.where((ct[:, 0, 0] == 1) & (ct[:, 0, 1] == 0), 0, 1).astype(np.int64)
    rows = data["sequence_lengths"].astype(np.int64) - sequence_lengths_offset
    return x, stat, arm, rows


def de_lists(x, u, arm, rows, n_arms=2):
    """Per-arm trajectory lists (X_a[L_i,1], U_a[L_i,U]) as handed to pysindy (utils.py:593-606)."""
    X = [[] for _ in range(n_arms)]
    U = [[] for _ in range(n_arms)]
    for i in range(x.shape[0]):
        L = int(rows[i])
        X[int(arm[i])].append(x[i, :L].reshape(-1, 1))
        U[int(arm[i])].append(np.repeat(u[i][None, :], L, axis=0))
    return X, U


# --------------------------------------------------------------------------------------
# A2 — derivative estimation (pysindy SmoothedFiniteDifference / FiniteDifference)
# --------------------------------------------------------------------------------------
# scipy.signal.savgol_filter(window_length=5, polyorder=3, mode='interp'):
# interior = savgol_coeffs(5,3); the 2+2 edge points are the least-squares cubic of the
# first/last 5 samples evaluated at the edge positions (scipy _fit_edge).
SAVGOL_5_3 = np.array([
    [69.0 / 70, 4.0 / 70, -6.0 / 70, 4.0 / 70, -1.0 / 70],     # position 0 of the window
    [2.0 / 35, 27.0 / 35, 12.0 / 35, -8.0 / 35, 2.0 / 35],     # position 1
    [-3.0 / 35, 12.0 / 35, 17.0 / 35, 12.0 / 35, -3.0 / 35],   # centre (interior)
    [2.0 / 35, -8.0 / 35, 12.0 / 35, 27.0 / 35, 2.0 / 35],     # position 3
    [-1.0 / 70, 4.0 / 70, -6.0 / 70, 4.0 / 70, 69.0 / 70],     # position 4
])

# pysindy FiniteDifference(d=1, order=4): 5-point central stencil in the interior; the
# first/last (n_stencil-1)//2 = 2 points use the one-sided 5-point (n_stencil_forward = d+order)
# stencil on the first/last 5 samples, evaluated at the endpoint (Vandermonde weights).
FD4 = np.array([
    [-25.0 / 12, 4.0, -3.0, 4.0 / 3, -1.0 / 4],                 # at sample 0 of t[0..4]
    [-1.0 / 4, -5.0 / 6, 3.0 / 2, -1.0 / 2, 1.0 / 12],          # at sample 1
    [1.0 / 12, -2.0 / 3, 0.0, 2.0 / 3, -1.0 / 12],              # centre
    [-1.0 / 12, 1.0 / 2, -3.0 / 2, 5.0 / 6, 1.0 / 4],           # at sample 3 of the last 5
    [1.0 / 4, -4.0 / 3, 3.0, -4.0, 25.0 / 12],                  # at sample 4 (last)
])


def _stencil5(x, W):
    """Apply a 5x5 edge/centre weight table along axis 0 (L >= 5)."""
    L = x.shape[0]
    if L < 5:
        raise ValueError("trajectory shorter than the 5-point stencil")
    y = np.empty_like(x)
    y[0] = W[0] @ x[0:5]
    y[1] = W[1] @ x[0:5]
    c = W[2]
    y[2:L - 2] = (c[0] * x[0:L - 4] + c[1] * x[1:L - 3] + c[2] * x[2:L - 2]
                  + c[3] * x[3:L - 1] + c[4] * x[4:L])
    y[L - 2] = W[3] @ x[L - 5:L]
    y[L - 1] = W[4] @ x[L - 5:L]
    return y


def savgol_5_3(x):
    return _stencil5(np.asarray(x, dtype=np.float64), SAVGOL_5_3)


def fd_order4(x, dt):
    return _stencil5(np.asarray(x, dtype=np.float64), FD4) / dt


def fd_order1(x, dt):
    """FiniteDifference(order=1): forward difference, backward at the last point."""
    x = np.asarray(x, dtype=np.float64)
    d = np.empty_like(x)
    d[:-1] = (x[1:] - x[:-1]) / dt
    d[-1] = (x[-1] - x[-2]) / dt
    return d


def smoothed_fd4(x, dt):
    """SmoothedFiniteDifference(savgol 5/3, order=4): returns (smoothed x, x_dot).  Only x_dot
    comes from the smoothed series: the library is evaluated on the RAW x (``build_regression``) —
    pinned by reproducing the reference's logged EQ_4_A..D equations to ~1e-15 on its own
    threefry cohorts (oracle/ref_cohort.py, tests/test_reference_cohort.py); evaluating the
    library on the smoothed x misses them by 3e-6..4e-5."""
    xs = savgol_5_3(x)
    return xs, fd_order4(xs, dt)


# --------------------------------------------------------------------------------------
# A3 — candidate library (pysindy PolynomialLibrary)
# --------------------------------------------------------------------------------------
def poly_library(n_inputs, degree=2, interaction_only=True, include_bias=True):
    """Exponent table [F, n_inputs] in pysindy column order (bias, linear, then products in
    ``itertools.combinations`` / ``combinations_with_replacement`` order per degree)."""
    comb = itertools.combinations if interaction_only else itertools.combinations_with_replacement
    exps = []
    for deg in range(0 if include_bias else 1, degree + 1):
        for c in comb(range(n_inputs), deg):
            e = [0] * n_inputs
            for i in c:
                e[i] += 1
            exps.append(e)
    return np.array(exps, dtype=np.int64)


def library_names(exps, input_names):
    names = []
    for e in exps:
        parts = []
        for i, k in enumerate(e):
            if k == 1:
                parts.append(input_names[i])
            elif k > 1:
                parts.append(f"{input_names[i]}^{k}")
        names.append(" ".join(parts) if parts else "1")
    return names


def eval_library(exps, Z):
    """Theta[R,F] for inputs Z[R,n_inputs] (state columns then control columns)."""
    Z = np.asarray(Z, dtype=np.float64)
    th = np.ones((Z.shape[0], exps.shape[0]))
    for j, e in enumerate(exps):
        for i, k in enumerate(e):
            for _ in range(int(k)):
                th[:, j] = th[:, j] * Z[:, i]
    return th


# --------------------------------------------------------------------------------------
# A4 — STLSQ (pysindy STLSQ; in-repo copy LSQIntialMask, pkpd/utils.py:213-327)
# --------------------------------------------------------------------------------------
def ridge_cholesky(X, y, alpha):
    """sklearn ``ridge_regression`` -> ``_solve_cholesky`` (_ridge.py:201-221):
    solve (X^T X + alpha I) w = X^T y with a Cholesky (posv) solve."""
    A = X.T @ X
    A.flat[::A.shape[0] + 1] += alpha
    Xy = X.T @ y
    Lc = np.linalg.cholesky(A)
    z = np.linalg.solve(Lc, Xy)
    return np.linalg.solve(Lc.T, z)


def stlsq(Theta, y, threshold, alpha, max_iter=100, unbias=True):
    """Returns (coef[F], ind[F], n_iter).  Semantics of pysindy 1.7 ``STLSQ._reduce``
    (restated in-repo at utils.py:256-327): initial support all ones (BaseOptimizer), ridge
    on the active columns, zero |c| < threshold (``_sparse_coefficients`` :213-219), stop when
    nothing was removed in the first pass or the support did not change (:308-310); empty
    support -> zeros (:275-281).  Then ind = |coef| > 1e-14 and the unbias refit (plain least
    squares on the support, pysindy ``_unbias``)."""
    F = Theta.shape[1]
    ind = np.ones(F, dtype=bool)
    n_selected0 = int(ind.sum())
    prev_pattern = np.ones(F, dtype=bool)          # history_[0] = lstsq guess (all non-zero)
    coef = np.zeros(F)
    it = 0
    for k in range(max_iter):
        it = k + 1
        if np.count_nonzero(ind) == 0:
            coef = np.zeros(F)
            break
        c_act = ridge_cholesky(Theta[:, ind], y, alpha)
        c = np.zeros(F)
        c[ind] = c_act
        big = np.abs(c) >= threshold
        c[~big] = 0.0
        coef = c
        ind = big
        pattern = coef != 0
        if int(ind.sum()) == n_selected0 or np.array_equal(pattern, prev_pattern):
            break
        prev_pattern = pattern
    ind = np.abs(coef) > SUPPORT_EPS
    if unbias and ind.any():
        out = np.zeros(F)
        out[ind] = np.linalg.lstsq(Theta[:, ind], y, rcond=None)[0]
        coef = out
    return coef, ind, it


def stlsq_initial_mask(Theta, y, threshold, alpha, init_coef, max_iter=100, unbias=True):
    """``LSQIntialMask`` (pkpd/utils.py:183-327) as used per patient by
    ``determine_individualized_equation_coefs`` (pkpd_simulation.py:791-800): the initial support is
    |global coef| > 1e-14 (:250-253), the stop rule compares the support size with the INITIAL one
    (:308) and the pattern with the previous history entry (:234-241; history_[0] is the full lstsq
    guess, all non-zero); then the unbias refit — unless sum|c| > 10, where the reference refits with
    unbias=False (:795-798), i.e. keeps the last thresholded ridge iterate.  Returns (coef, ind, it)."""
    F = Theta.shape[1]
    init = np.abs(np.asarray(init_coef, dtype=np.float64)) > SUPPORT_EPS
    ind = init.copy()
    n_sel0 = int(init.sum())
    prev_pattern = np.ones(F, dtype=bool)
    coef = np.zeros(F)
    it = 0
    for k in range(max_iter):
        it = k + 1
        if not ind.any():
            coef = np.zeros(F)
            break
        c_act = ridge_cholesky(Theta[:, ind], y, alpha)
        c = np.zeros(F)
        c[ind] = c_act
        big = np.abs(c) >= threshold
        c[~big] = 0.0
        coef = c
        ind = big
        pattern = coef != 0
        if int(ind.sum()) == n_sel0 or np.array_equal(pattern, prev_pattern):
            break
        prev_pattern = pattern
    ridge = coef
    sup = np.abs(coef) > SUPPORT_EPS
    if unbias and sup.any():
        out = np.zeros(F)
        out[sup] = np.linalg.lstsq(Theta[:, sup], y, rcond=None)[0]
        if np.abs(out).sum() > 10.0:
            out = ridge
        coef = out
    return coef, np.abs(coef) > SUPPORT_EPS, it


def per_patient_fit(x, u, arm, rows, dt, exps, global_coef, threshold, alpha, max_iter=100, fd="smoothed4"):
    """Per-patient refit: every patient with >= 5 rows refits its own
    arm's equation on its own rows with the initial support of the global model
    (``stlsq_initial_mask``); the other arms keep the global coefficients.  Patients with < 5 rows
    keep the global model (pysindy would raise).  Returns coef[N, A, F], mask[N, F], iters[N]."""
    N = x.shape[0]
    A, F = global_coef.shape
    coef = np.repeat(np.asarray(global_coef, dtype=np.float64)[None], N, axis=0)
    mask = np.zeros((N, F), dtype=np.int8)
    iters = np.zeros(N, dtype=np.int32)
    for i in range(N):
        a = int(arm[i])
        L = int(rows[i])
        if L < 5:
            mask[i] = np.abs(global_coef[a]) > SUPPORT_EPS
            continue
        Z, Y = build_regression([x[i, :L].reshape(-1, 1)], [np.repeat(u[i][None, :], L, 0)], dt, fd)
        c, ind, it = stlsq_initial_mask(eval_library(exps, Z), Y, threshold, alpha, global_coef[a], max_iter)
        coef[i, a] = c
        mask[i] = ind
        iters[i] = it
    return coef, mask, iters


def stlsq_gram(G, b, threshold, alpha, max_iter=100, unbias=True):
    """The same algorithm expressed on the Gram G = Theta^T Theta and moment b = Theta^T y
    (the form the GPU path uses; unbias via the normal equations)."""
    F = G.shape[0]
    ind = np.ones(F, dtype=bool)
    prev_pattern = np.ones(F, dtype=bool)
    coef = np.zeros(F)
    it = 0
    for k in range(max_iter):
        it = k + 1
        if not ind.any():
            coef = np.zeros(F)
            break
        S = np.nonzero(ind)[0]
        A = G[np.ix_(S, S)] + alpha * np.eye(S.size)
        c = np.zeros(F)
        c[S] = np.linalg.solve(A, b[S])
        big = np.abs(c) >= threshold
        c[~big] = 0.0
        coef = c
        ind = big
        pattern = coef != 0
        if int(ind.sum()) == F or np.array_equal(pattern, prev_pattern):
            break
        prev_pattern = pattern
    ind = np.abs(coef) > SUPPORT_EPS
    if unbias and ind.any():
        # the unbias is lstsq's minimum-norm solution: exactly duplicated support columns (||theta_i -
        # theta_k||^2 = G_ii + G_kk - 2 G_ik = 0, b_i = b_k; e.g. a static equal to 1 for every patient,
        # EQ_5_A/B) are solved once and their coefficient split equally (the GPU solvers do the same)
        S = list(np.nonzero(ind)[0])
        rep = {}
        for k in S:
            for i in S:
                if i >= k:
                    break
                if rep.get(i, i) == i and G[i, i] == G[k, k] and G[k, i] == G[i, i] and b[i] == b[k]:
                    rep[k] = i
                    break
        R_ = [k for k in S if rep.get(k, k) == k]
        out = np.zeros(F)
        out[R_] = np.linalg.solve(G[np.ix_(R_, R_)], b[R_])
        for i in R_:
            grp = [k for k in S if rep.get(k, k) == i]
            out[grp] = out[i] / len(grp)
        coef = out
    return coef, ind, it


# --------------------------------------------------------------------------------------
# SINDy.fit equivalent (sindy.py:190-192) — multiple trajectories, per arm
# --------------------------------------------------------------------------------------
def build_regression(X_list, U_list, dt, fd="smoothed4"):
    """Concatenate per-trajectory rows (multiple_trajectories=True): library inputs [x, u] with
    the RAW x (also for SmoothedFiniteDifference, whose smoothing only feeds x_dot — pinned, see
    ``smoothed_fd4``) and targets x_dot."""
    Z, Y = [], []
    for X, U in zip(X_list, U_list):
        x = X[:, 0]
        if fd == "smoothed4":
            _, xd = smoothed_fd4(x, dt)
        elif fd == "order4":
            xd = fd_order4(x, dt)
        elif fd == "order1":
            xd = fd_order1(x, dt)
        else:
            raise ValueError(fd)
        Z.append(np.concatenate([x[:, None], U], axis=1))
        Y.append(xd)
    return np.concatenate(Z, axis=0), np.concatenate(Y, axis=0)


def sindy_fit(X_list, U_list, dt, threshold=0.1, alpha=0.5, max_iter=100, fd="smoothed4",
              degree=2, interaction_only=True):
    n_inputs = 1 + U_list[0].shape[1]
    exps = poly_library(n_inputs, degree, interaction_only)
    Z, Y = build_regression(X_list, U_list, dt, fd)
    Theta = eval_library(exps, Z)
    coef, ind, it = stlsq(Theta, Y, threshold, alpha, max_iter)
    return coef, ind, exps, it


def gram_moments(x, u, arm, rows, dt, exps, n_arms=2, fd="smoothed4"):
    """Per-arm Gram G[A,F,F] and moment b[A,F] over all rows (sum over patients of
    Theta_p^T Theta_p, Theta_p^T x_dot_p) — what ``insite_gram_f64`` returns."""
    F = exps.shape[0]
    G = np.zeros((n_arms, F, F))
    b = np.zeros((n_arms, F))
    for i in range(x.shape[0]):
        L = int(rows[i])
        if L < 5:
            continue
        Zi, Yi = build_regression([x[i, :L].reshape(-1, 1)], [np.repeat(u[i][None, :], L, 0)], dt, fd)
        th = eval_library(exps, Zi)
        G[int(arm[i])] += th.T @ th
        b[int(arm[i])] += th.T @ Yi
    return G, b


def gram_moments_vectorized(x, u, arm, rows_const, dt, exps, n_arms=2):
    """Vectorised variant for equal row counts (CPU baseline timing); smoothed FD4, library on
    the raw x."""
    L = int(rows_const)
    X = x[:, :L]
    xs = np.empty_like(X)
    W = SAVGOL_5_3
    xs[:, 0] = X[:, :5] @ W[0]
    xs[:, 1] = X[:, :5] @ W[1]
    c = W[2]
    xs[:, 2:L - 2] = c[0] * X[:, 0:L - 4] + c[1] * X[:, 1:L - 3] + c[2] * X[:, 2:L - 2] + c[3] * X[:, 3:L - 1] + c[4] * X[:, 4:L]
    xs[:, L - 2] = X[:, L - 5:] @ W[3]
    xs[:, L - 1] = X[:, L - 5:] @ W[4]
    D = np.empty_like(X)
    W = FD4
    D[:, 0] = xs[:, :5] @ W[0]
    D[:, 1] = xs[:, :5] @ W[1]
    c = W[2]
    D[:, 2:L - 2] = c[0] * xs[:, 0:L - 4] + c[1] * xs[:, 1:L - 3] + c[3] * xs[:, 3:L - 1] + c[4] * xs[:, 4:L]
    D[:, L - 2] = xs[:, L - 5:] @ W[3]
    D[:, L - 1] = xs[:, L - 5:] @ W[4]
    D /= dt
    F = exps.shape[0]
    G = np.zeros((n_arms, F, F))
    b = np.zeros((n_arms, F))
    for a in range(n_arms):
        sel = arm == a
        Z = np.concatenate([X[sel].reshape(-1, 1), np.repeat(u[sel], L, axis=0)], axis=1)
        th = eval_library(exps, Z)
        G[a] = th.T @ th
        b[a] = th.T @ D[sel].reshape(-1)
    return G, b


# --------------------------------------------------------------------------------------
# Joint ("one ODE") model — ABLATION_ONE_ODE (run.py:198-201: joint_model=true, multilabel treatments)
# --------------------------------------------------------------------------------------
def de_format_joint(data, scaling_params, sequence_lengths_offset=1):
    """The joint branch of ``process_dataset_into_de_format`` (pkpd/utils.py:639-672, 486-497): per patient
    X = unscaled_outputs[:L] (the OUTPUTS V[1:], not the reconstructed series), U = concat(treatments[:L],
    statics[:L]) with the multilabel (binary) treatments, L = seq_len - offset (1 for EQ_4, 0 for
    cancer_sim / EQ_5).  Returns x [N, T-1], inputs [N, T-1, n_in] (0/1), statics [N, U], rows [N]."""
    _, stat = unscale_inputs(data, scaling_params)
    x = data["unscaled_outputs"][..., 0]
    inputs = np.asarray(data["current_treatments"], dtype=np.float64)
    rows = data["sequence_lengths"].astype(np.int64) - sequence_lengths_offset
    return x, inputs, stat, rows


def build_regression_joint(x, inputs, stat, rows, dt, fd="smoothed4"):
    """Concatenated joint regression rows: library inputs [x, inputs_k, statics], targets x_dot (pysindy
    multiple_trajectories over the patients; the raw x in the library, x_dot by ``fd``)."""
    X = [x[i, :int(rows[i])].reshape(-1, 1) for i in range(x.shape[0]) if int(rows[i]) >= (5 if "4" in fd else 2)]
    U = [np.concatenate([inputs[i, :int(rows[i])], np.repeat(stat[i][None, :], int(rows[i]), 0)], axis=1)
         for i in range(x.shape[0]) if int(rows[i]) >= (5 if "4" in fd else 2)]
    if fd == "smoothed1" or fd == "order1":
        from . import segments_ref as SG
        Z, Y = [], []
        for Xi, Ui in zip(X, U):
            zi, yi = SG.derivative(Xi[:, 0], dt, fd)
            Z.append(np.concatenate([zi[:, None], Ui], axis=1))
            Y.append(yi)
        return np.concatenate(Z), np.concatenate(Y)
    return build_regression(X, U, dt, fd)


def rollout_inputs(y0, stat, inputs, coef, exps, dt, method="euler5", substeps=None):
    """Open-loop rollout of a model whose library has per-step inputs (the joint model's
    pred_dy_dt = mod_0(x0=y, u0=treatment_k, u1.. = statics), sindy.py:283-288, 317-322): step k evaluates
    the RHS on u_k = [inputs[:, k], statics].  coef [F] (the joint model's single row)."""
    N, T = inputs.shape[:2]
    y = np.asarray(y0, dtype=np.float64).copy()
    out = np.empty((N, T))
    cr = np.repeat(np.asarray(coef, dtype=np.float64)[None, :], N, axis=0)
    for k in range(T):
        uk = np.concatenate([inputs[:, k], stat], axis=1)
        if method in ("euler5", "euler"):
            n_sub = STEPS_FOR_DT if method == "euler5" else int(substeps or 1)
            h = dt / n_sub
            for _ in range(n_sub):
                y = y + rhs_literal(y, uk, cr, exps) * h
        else:
            n_sub = int(substeps or 1)
            h = dt / n_sub
            for _ in range(n_sub):
                k1 = rhs_literal(y, uk, cr, exps)
                k2 = rhs_literal(y + 0.5 * h * k1, uk, cr, exps)
                k3 = rhs_literal(y + 0.5 * h * k2, uk, cr, exps)
                k4 = rhs_literal(y + h * k3, uk, cr, exps)
                y = y + (h / 6.0) * (k1 + 2.0 * k2 + 2.0 * k3 + k4)
        out[:, k] = y
    return out


# --------------------------------------------------------------------------------------
# A6 — model -> RHS and global_equation_string (pkpd/utils.py:372-397; sindy.py:272-282)
# --------------------------------------------------------------------------------------
def equation_terms(coefs, names, quantize=False, round_to=3):
    """Term string of ``convert_sindy_model_to_sympyjax_model_core`` (utils.py:377-391)."""
    s = ""
    for j, c in enumerate(np.asarray(coefs, dtype=np.float64)):
        if np.abs(c) > RHS_COEF_EPS:
            if quantize:
                c = np.round(c, round_to)
            s += f"+{c}*" + names[j].replace(" ", "*")
    return s


def global_equation_string(joint_coefs, names):
    """``f'Treatment 0: x_dot = {str_0} | Treatment 1: x_dot = {str_1}'`` (sindy.py:276)."""
    return " | ".join(f"Treatment {a}: x_dot = {equation_terms(c, names)}" for a, c in enumerate(joint_coefs))


# --------------------------------------------------------------------------------------
# A7/A8 — integrators and the batched rollout (utils.py:68-94; sindy.py:371-431, 767-778)
# --------------------------------------------------------------------------------------
def rhs_literal(y, u, coef_rows, exps):
    """sum_j c_j * Theta_j(y, u) over terms with |c_j| > 1e-3 (utils.py:388), evaluated
    literally per column in library order.  y[N], u[N,U], coef_rows[N,F]."""
    acc = np.zeros_like(y)
    for j, e in enumerate(exps):
        c = coef_rows[:, j]
        keep = np.abs(c) > RHS_COEF_EPS
        if not keep.any():
            continue
        th = np.ones_like(y)
        for _ in range(int(e[0])):
            th = th * y
        for i in range(1, e.shape[0]):
            for _ in range(int(e[i])):
                th = th * u[:, i - 1]
        acc = acc + np.where(keep, c, 0.0) * th
    return acc


def rollout(y0, u, arm, coef, exps, dt, method="euler5", substeps=None):
    """Open-loop rollout of every row over T steps; output y[N,T] = state after each step.

    ``coef`` is [A,F] (global model) or [N,A,F] (per-patient, C4 / predict_with_reduced_coefs).
    euler5: per observation interval, 5 forward-Euler sub-steps y <- y + f(y)*h, h = dt/5
    (utils.py:68-79, 86-90, called at sindy.py:421).  rk4: classical RK4 with ``substeps``
    (default 1) steps per interval.  euler: ``substeps`` Euler steps (1 = standard resolution,
    utils.py:81-84)."""
    y = np.asarray(y0, dtype=np.float64).copy()
    N, T = arm.shape
    out = np.empty((N, T))
    per_patient = coef.ndim == 3
    rowsel = np.arange(N)
    for k in range(T):
        a = arm[:, k].astype(np.int64)
        cr = coef[rowsel, a] if per_patient else coef[a]
        if method in ("euler5", "euler"):
            n_sub = STEPS_FOR_DT if method == "euler5" else int(substeps or 1)
            h = dt / n_sub
            for _ in range(n_sub):
                y = y + rhs_literal(y, u, cr, exps) * h
        elif method == "rk4":
            n_sub = int(substeps or 1)
            h = dt / n_sub
            for _ in range(n_sub):
                k1 = rhs_literal(y, u, cr, exps)
                k2 = rhs_literal(y + 0.5 * h * k1, u, cr, exps)
                k3 = rhs_literal(y + 0.5 * h * k2, u, cr, exps)
                k4 = rhs_literal(y + h * k3, u, cr, exps)
                y = y + (h / 6.0) * (k1 + 2.0 * k2 + 2.0 * k3 + k4)
        else:
            raise ValueError(method)
        out[:, k] = y
    return out


def odeint_euler5(f, y0, t):
    """Restatement of the reference ``odeint`` (utils.py:86-94) for scalar f(y, t):
    5 sub-steps per interval when hmax < dt, else one Euler step per interval."""
    t = np.asarray(t, dtype=np.float64)
    dts = np.diff(t)
    ys = [np.float64(y0)]
    y = np.float64(y0)
    high = HMAX < dts[0]
    for d in dts:
        if high:
            h = d / STEPS_FOR_DT
            for _ in range(STEPS_FOR_DT):
                y = y + f(y, h) * h
        else:
            y = y + f(y, d) * d
        ys.append(y)
    return np.array(ys)


# --------------------------------------------------------------------------------------
# A9 / A10 — autoregressive slice and metrics (sindy.py:717-760; time_varying_model.py:236-313)
# --------------------------------------------------------------------------------------
def autoregressive_slice(pred, seq_len, tau, offset=1):
    """jax.lax.dynamic_slice(pred, (i, max(1, sl - tau), 0), (1, tau, 1)) with JAX's clamp."""
    N, T = pred.shape[:2]
    out = np.empty((N, tau) + pred.shape[2:])
    for i in range(N):
        lo = max(offset, int(seq_len[i]) - tau)
        lo = min(max(lo, 0), T - tau)
        out[i] = pred[i, lo:lo + tau]
    return out


def masked_rmse(pred_unscaled, target_unscaled, active, norm_const=MAX_VALUE, percentage=True,
                one_step_counterfactual=False):
    mse = ((pred_unscaled - target_unscaled) ** 2) * active
    mse_orig = (mse.sum(0).sum(-1) / active.sum(0).sum(-1)).mean()
    orig = np.sqrt(mse_orig) / norm_const
    mse_all = mse.sum() / active.sum()
    allv = np.sqrt(mse_all) / norm_const
    scale = 100.0 if percentage else 1.0
    if not one_step_counterfactual:
        return orig * scale, allv * scale
    n, t, o = active.shape
    last = active - np.concatenate([active[:, 1:, :], np.zeros((n, 1, o))], axis=1)
    mse_last = (((pred_unscaled - target_unscaled) ** 2) * last).sum() / last.sum()
    return orig * scale, allv * scale, np.sqrt(mse_last) / norm_const * scale


def n_step_rmses(pred_unscaled, target_unscaled, active, norm_const=MAX_VALUE, percentage=True):
    mse = ((pred_unscaled - target_unscaled) ** 2) * active
    mse_orig = mse.sum(0).sum(-1) / active.sum(0).sum(-1)
    r = np.sqrt(mse_orig) / norm_const
    return r * (100.0 if percentage else 1.0)


# --------------------------------------------------------------------------------------
# End-to-end: train_sindy.main equivalent (runnables/train_sindy.py:21-113), SINDy backbone
# --------------------------------------------------------------------------------------
def sindy_pipeline(coll, threshold=0.1, alpha=0.5, dt=None, method="euler5", joint_model=False, degree=2,
                   interaction_only=True):
    """train_sindy.main for the EQ_4 SINDy backbone: per-arm fits (default), the degree-4 ablation library
    (``degree=4, interaction_only=False``, sindy.py:185-186) or the joint model (``joint_model``: one fit
    with the multilabel treatment as library input u0, pkpd/utils.py:486-497, on a multilabel collection)."""
    train = coll["train"]
    T = train.data["prev_outputs"].shape[1] + 1
    dt = MAX_TIME_HORIZON / T if dt is None else dt
    if joint_model:
        x, inputs, stat, rows = de_format_joint(train.data, train.scaling_params)
        n_in = inputs.shape[-1]
        exps = poly_library(1 + n_in + stat.shape[1], degree, interaction_only)
        names = library_names(exps, ["x0"] + [f"u{i}" for i in range(n_in + stat.shape[1])])
        Z, Y = build_regression_joint(x, inputs, stat, rows, dt)
        c, _, _ = stlsq(eval_library(exps, Z), Y, threshold, alpha)
        joint = c[None, :]
        res = {"joint_coefs": joint, "global_equation_string": f"Joint Model: x_dot = {equation_terms(c, names)}"}

        def predict(sub):
            prev, st = unscale_inputs(sub.data, sub.scaling_params)
            return rollout_inputs(prev[:, 0], st, np.asarray(sub.data["current_treatments"], dtype=np.float64), c,
                                  exps, dt, method)
    else:
        x, u, arm, rows = de_format(train.data, train.scaling_params)
        X, U = de_lists(x, u, arm, rows)
        exps = poly_library(3, degree, interaction_only)
        names = library_names(exps, ["x0", "u0", "u1"])
        coefs = []
        for a in range(2):
            c, _, _, _ = sindy_fit(X[a], U[a], dt, threshold, alpha, degree=degree, interaction_only=interaction_only)
            coefs.append(c)
        joint = np.stack(coefs)
        res = {"joint_coefs": joint, "global_equation_string": global_equation_string(joint, names)}

        def predict(sub):
            prev, stat = unscale_inputs(sub.data, sub.scaling_params)
            arms = np.argmax(sub.data["current_treatments"], axis=-1)
            return rollout(prev[:, 0], stat, arms, joint, exps, dt, method)

    one = coll.get("test_cf_one_step")
    if one is not None:
        pu = predict(one)
        o, a_, l = masked_rmse(pu[..., None], one.data["unscaled_outputs"], one.data["active_entries"],
                               one_step_counterfactual=True)
        res.update(encoder_test_rmse_orig=o, encoder_test_rmse_all=a_, encoder_test_rmse_last=l)
    seqs = coll.get("test_cf_treatment_seq")
    if seqs is not None:
        pu = predict(seqs)
        tau = seqs.data_processed_seq["outputs"].shape[1]
        sl = autoregressive_slice(pu[..., None], seqs.data["sequence_lengths"], tau)
        r = n_step_rmses(sl, seqs.data_processed_seq["unscaled_outputs"], seqs.data_processed_seq["active_entries"])
        for k, v in enumerate(r):
            res[f"decoder_test_rmse_{k + 2}-step"] = v
    return res


def euler5_rate_known_answer(c, dt=STANDARD_DT):
    """Continuous rate whose exact exponential matches one Euler-5 interval of -c*y:
    ln(1 - c*h)/(h*c) with h = dt/5 (e.g. 30*ln(1-c/30)/c at dt = 1/6)."""
    h = dt / STEPS_FOR_DT
    return np.log1p(-c * h) / (h * c)
