"""cancer_sim_ref — CPU restatement of the reference's cancer_sim (Geng et al. tumour growth) cohort
generator, with the reference's numpy legacy-RNG draw order — TEST INFRASTRUCTURE ONLY (imported by
``tests/`` and tools that regenerate golden fixtures, never by the product package).

Why: the F4 (cancer_sim / EQ_5 treatment-segment) oracle ``segments_ref`` was pinned only to scipy
primitives.  The reference seeds the cancer_sim collection with ``np.random.seed(seed)``
(``libs_m/ct/src/data/cancer_sim/dataset.py:589``) and every subset then draws from numpy's global
``RandomState`` in a fixed order, so with the same draw order the published cohorts -- and through
them the published equations and metrics (``results/2_main_table/final_with_insite.txt:6``,
``results/ablation/one_ode/build_tables/...one_big_ode.txt``) -- are reproducible here.  Draws go
through an explicit ``np.random.RandomState(seed)`` (the stream of the seeded global state); scipy's
``truncnorm.rvs`` is called with that state as ``random_state``.

Restated (reference file:line, ``libs_m/ct/src/data/cancer_sim/``):
* ``calc_volume`` / ``calc_diameter`` and the constants (``cancer_simulation.py:34-60``);
* ``get_standard_params`` (``:96-215``): stage draw ``choice(p=...)``, per-stage truncated-normal log
  diameters (stages in sorted order), correlated (alpha, rho) by ``multivariate_normal`` with
  rejection, patient types, truncated-normal beta_c, final ``shuffle``;
* ``generate_params`` (``:66-93``): sigmoid intercepts/betas from chemo/radio coefficients;
* ``simulate_factual`` (``:218-375``): the per-patient volume recursion with dosages, 15-day
  window mean diameter -> sigmoid assignment, death / recovery stopping;
* ``get_scaling_params`` (``:776-796``) and ``SyntheticCancerDataset.process_data`` (``dataset.py:96-185``,
  multiclass and multilabel treatments);
* the collection's draw order (``dataset.py:556-605``): train, val (factual), test one-step and
  test tau-step counterfactual subsets, all from the one seeded stream.
"""
from __future__ import annotations

import numpy as np
from scipy.stats import truncnorm


def calc_volume(diameter):
    return 4 / 3 * np.pi * (diameter / 2) ** 3


def calc_diameter(volume):
    return ((volume / (4 / 3 * np.pi)) ** (1 / 3)) * 2


TUMOUR_CELL_DENSITY = 5.8 * 10 ** 8
TUMOUR_DEATH_THRESHOLD = calc_volume(13)
TUMOUR_SIZE_DISTRIBUTIONS = {"I": (1.72, 4.70, 0.3, 5.0), "II": (1.96, 1.63, 0.3, 13.0), "IIIA": (1.91, 9.40, 0.3, 13.0),
                             "IIIB": (2.76, 6.87, 0.3, 13.0), "IV": (3.86, 8.82, 0.3, 13.0)}
CANCER_STAGE_OBSERVATIONS = {"I": 1432, "II": 128, "IIIA": 1306, "IIIB": 7248, "IV": 12840}


def get_standard_params(num_patients, rs, equation=None):
    """cancer_simulation.py:96-215 with the draws taken from RandomState ``rs`` in the reference order.
    ``equation`` "EQ_5_A".."EQ_5_D": the continuous variant (continuous.py:98-224): patient type always 1
    for A / B (:178-181), the truncated-normal beta_c draw only for D (:195-201)."""
    total = sum(CANCER_STAGE_OBSERVATIONS.values())
    props = {k: CANCER_STAGE_OBSERVATIONS[k] / total for k in CANCER_STAGE_OBSERVATIONS}
    stages = sorted(TUMOUR_SIZE_DISTRIBUTIONS)
    initial_stages = rs.choice(stages, num_patients, p=[props[k] for k in stages])
    diam, sim_stages = [], []
    for stg in stages:
        count = int(np.sum((initial_stages == stg) * 1))
        mu, sigma, lb, ub = TUMOUR_SIZE_DISTRIBUTIONS[stg]
        lo = (np.log(lb) - mu) / sigma
        hi = (np.log(ub) - mu) / sigma
        rvs = truncnorm.rvs(lo, hi, size=count, random_state=rs)
        diam += list(np.exp(rvs * sigma + mu))
        sim_stages += [stg] * count
    K = calc_volume(30)
    alpha_beta_ratio = 10
    alpha_rho_corr = 0.87
    lower, upper = 0.0, np.inf
    rho_params = (7 * 10 ** -5, 7.23 * 10 ** -3)
    alpha_params = (0.0398, 0.168)
    beta_c_params = (0.028, 0.0007)
    cov = np.array([[alpha_params[1] ** 2, alpha_rho_corr * alpha_params[1] * rho_params[1]],
                    [alpha_rho_corr * alpha_params[1] * rho_params[1], rho_params[1] ** 2]])
    mean = np.array([alpha_params[0], rho_params[0]])
    sim = []
    while len(sim) < num_patients:
        holder = rs.multivariate_normal(mean, cov, size=num_patients)
        for i in range(holder.shape[0]):
            if holder[i, 0] > lower and holder[i, 1] > lower:
                sim.append(holder[i, :])
    patient_types = rs.choice([1] if equation in ("EQ_5_A", "EQ_5_B") else [1, 2, 3], num_patients)
    chemo_adj = np.array([0.0 if i < 3 else 0.1 for i in patient_types])
    radio_adj = np.array([0.0 if i > 1 else 0.1 for i in patient_types])
    sim = np.array(sim)[:num_patients, :]
    alpha = sim[:, 0] + alpha_params[0] * radio_adj
    rho = sim[:, 1]
    beta = alpha / alpha_beta_ratio
    if equation is None or equation == "EQ_5_D":
        beta_c = beta_c_params[0] + beta_c_params[1] * truncnorm.rvs(
            (lower - beta_c_params[0]) / beta_c_params[1], (upper - beta_c_params[0]) / beta_c_params[1],
            size=num_patients, random_state=rs) + beta_c_params[0] * chemo_adj
    else:
        beta_c = beta_c_params[0] + beta_c_params[0] * chemo_adj
    holder = {"patient_types": patient_types, "initial_stages": np.array(sim_stages),
              "initial_volumes": calc_volume(np.array(diam)), "alpha": alpha, "rho": rho, "beta": beta,
              "beta_c": beta_c, "K": np.array([K for _ in range(num_patients)])}
    idx = [i for i in range(num_patients)]
    rs.shuffle(idx)
    return {k: v[idx] for k, v in holder.items()}


def generate_params(num_patients, chemo_coeff, radio_coeff, window_size, lag, rs, equation=None):
    """cancer_simulation.py:66-93 (continuous.py:68-95)."""
    p = get_standard_params(num_patients, rs, equation)
    n = len(p["patient_types"])
    d_max = calc_diameter(TUMOUR_DEATH_THRESHOLD)
    p["chemo_sigmoid_intercepts"] = np.full(n, d_max / 2.0)
    p["radio_sigmoid_intercepts"] = np.full(n, d_max / 2.0)
    p["chemo_sigmoid_betas"] = np.full(n, chemo_coeff / d_max)
    p["radio_sigmoid_betas"] = np.full(n, radio_coeff / d_max)
    p["window_size"] = window_size
    p["lag"] = lag
    p["equation"] = equation
    return p


def _observation_noise(V, p, rs):
    """EQ_5_B/C/D: 0.01 * N(0, 1) added to the whole volume array after the simulation (continuous.py:366-367,
    568-569, 784-785); cancer_sim and EQ_5_A are noise-free."""
    eq = p.get("equation")
    if eq is not None and eq.split("_")[-1] in ("B", "C", "D"):
        return V + 0.01 * rs.normal(size=V.shape)
    return V


def _assign_prob(p, i, volumes_used):
    """Sigmoid assignment probabilities on the window-mean diameter (cancer_simulation.py:301-317)."""
    metric = np.array([calc_diameter(v) for v in volumes_used]).mean()
    radio = 1.0 / (1.0 + np.exp(-p["radio_sigmoid_betas"][i] * (metric - p["radio_sigmoid_intercepts"][i])))
    chemo = 1.0 / (1.0 + np.exp(-p["chemo_sigmoid_betas"][i] * (metric - p["chemo_sigmoid_intercepts"][i])))
    return chemo, radio


def simulate_factual(p, seq_length, rs):
    """cancer_simulation.py:218-375 (no assigned actions)."""
    radio_amt, chemo_amt, half_life = 2.0, 5.0, 1
    window, lag = p["window_size"], p["lag"]
    N = p["initial_stages"].shape[0]
    V = np.zeros((N, seq_length))
    chemo_d = np.zeros((N, seq_length))
    radio_d = np.zeros((N, seq_length))
    chemo_a = np.zeros((N, seq_length))
    radio_a = np.zeros((N, seq_length))
    sl = np.zeros(N)
    death = np.zeros((N, seq_length))
    recov = np.zeros((N, seq_length))
    chemo_p = np.zeros((N, seq_length))
    radio_p = np.zeros((N, seq_length))
    noise_terms = 0.01 * rs.randn(N, seq_length)
    recovery_rvs = rs.rand(N, seq_length)
    chemo_rvs = rs.rand(N, seq_length)
    radio_rvs = rs.rand(N, seq_length)
    for i in range(N):
        noise = noise_terms[i]
        V[i, 0] = p["initial_volumes"][i]
        alpha, beta, beta_c, rho, K = p["alpha"][i], p["beta"][i], p["beta_c"][i], p["rho"][i], p["K"][i]
        b_death = b_recover = False
        for t in range(1, seq_length - 1):
            V[i, t] = V[i, t - 1] * (1 + rho * np.log(K / V[i, t - 1]) - beta_c * chemo_d[i, t - 1]
                                     - (alpha * radio_d[i, t - 1] + beta * radio_d[i, t - 1] ** 2) + noise[t])
            cur_chemo = 0.0
            prev_chemo = 0.0 if t == 0 else chemo_d[i, t - 1]
            used = V[i, max(t - window - lag, 0):max(t - lag, 0)] if t >= lag else np.zeros((1,))
            chemo_prob, radio_prob = _assign_prob(p, i, used)
            chemo_p[i, t] = chemo_prob
            radio_p[i, t] = radio_prob
            if radio_rvs[i, t] < radio_prob:
                radio_a[i, t] = 1
                radio_d[i, t] = radio_amt
            if chemo_rvs[i, t] < chemo_prob:
                chemo_a[i, t] = 1
                cur_chemo = chemo_amt
            chemo_d[i, t] = prev_chemo * np.exp(-np.log(2) / half_life) + cur_chemo
            if V[i, t] > TUMOUR_DEATH_THRESHOLD:
                V[i, t] = TUMOUR_DEATH_THRESHOLD
                b_death = True
                break
            if recovery_rvs[i, t] < np.exp(-V[i, t] * TUMOUR_CELL_DENSITY):
                V[i, t] = 0
                b_recover = True
                break
        sl[i] = int(t + 1)
        death[i, t] = 1 if b_death else 0
        recov[i, t] = 1 if b_recover else 0
    V = _observation_noise(V, p, rs)
    return {"cancer_volume": V, "chemo_dosage": chemo_d, "radio_dosage": radio_d, "chemo_application": chemo_a,
            "radio_application": radio_a, "chemo_probabilities": chemo_p, "radio_probabilities": radio_p,
            "sequence_lengths": sl, "death_flags": death, "recovery_flags": recov,
            "patient_types": p["patient_types"]}


def get_scaling_params(sim):
    """cancer_simulation.py:776-796: means / stds over active entries (np.mean / np.std of the
    concatenated python lists) plus the static patient types.  Returns (mean, std) dicts."""
    means, stds = {}, {}
    sl = sim["sequence_lengths"]
    for k in ("cancer_volume", "chemo_dosage", "radio_dosage"):
        vals = []
        for i in range(sl.shape[0]):
            vals += list(sim[k][i, :int(sl[i])])
        means[k] = np.mean(vals)
        stds[k] = np.std(vals)
    means["patient_types"] = np.mean(sim["patient_types"])
    stds["patient_types"] = np.std(sim["patient_types"])
    return means, stds


def process_data(sim, scaling, treatment_mode="multiclass", equation=None, include_continuous_treatment=False):
    """SyntheticCancerDataset.process_data (dataset.py:96-185) for one-step-ahead data (continuous
    dataset.py:96-200: EQ_5_A / B set the patient-type std to 1, their single type has std 0).
    ``include_continuous_treatment`` (what train_sindy.py:41-42 passes for every EQ_5 dataset): the scaled
    chemo dosage is a third covariate channel, so static_features = [patient type, chemo dosage at t = 0]
    and the model's dim_static_features becomes 2 (train_sindy.py:48)."""
    mean, std = dict(scaling[0]), dict(scaling[1])
    if equation in ("EQ_5_A", "EQ_5_B"):
        std["patient_types"] = 1
    offset = horizon = 1
    for k in ("chemo_application", "radio_application"):
        mean[k], std[k] = 0, 1
    keys = ("cancer_volume", "patient_types") + (("chemo_dosage",) if include_continuous_treatment else ()) + \
        ("chemo_application", "radio_application")
    input_means = np.array([mean[k] for k in keys], dtype=np.float64)
    input_stds = np.array([std[k] for k in keys], dtype=np.float64)
    data = dict(sim)
    cv = (sim["cancer_volume"] - mean["cancer_volume"]) / std["cancer_volume"]
    pt = (sim["patient_types"] - mean["patient_types"]) / std["patient_types"]
    pt = np.stack([pt for _ in range(cv.shape[1])], axis=1)
    treatments = np.concatenate([sim["chemo_application"][:, :-offset, None], sim["radio_application"][:, :-offset, None]],
                                axis=-1)
    if treatment_mode == "multiclass":
        code = (treatments[..., 0] + 2 * treatments[..., 1]).astype(np.int64)   # [0,0]->0 [1,0]->1 [0,1]->2 [1,1]->3
        one_hot = np.zeros(treatments.shape[:2] + (4,))
        np.put_along_axis(one_hot, code[..., None], 1.0, axis=-1)
        data["prev_treatments"] = one_hot[:, :-1, :]
        data["current_treatments"] = one_hot
    elif treatment_mode == "multilabel":
        data["prev_treatments"] = treatments[:, :-1, :]
        data["current_treatments"] = treatments
    else:
        raise ValueError(treatment_mode)
    cov = [cv[:, :-offset, None], pt[:, :-offset, None]]
    if include_continuous_treatment:
        cd = (sim["chemo_dosage"] - mean["chemo_dosage"]) / std["chemo_dosage"]
        cov.append(cd[:, :-offset, None])
    cov = np.concatenate(cov, axis=-1)
    outputs = cv[:, horizon:, None]
    active = np.zeros(outputs.shape)
    for i in range(sim["sequence_lengths"].shape[0]):
        active[i, :int(sim["sequence_lengths"][i]), :] = 1
    data["current_covariates"] = cov
    data["outputs"] = outputs
    data["active_entries"] = active
    data["unscaled_outputs"] = outputs * std["cancer_volume"] + mean["cancer_volume"]
    scaling_params = {"input_means": input_means, "inputs_stds": input_stds,
                      "output_means": mean["cancer_volume"], "output_stds": std["cancer_volume"]}
    data["prev_outputs"] = cov[:, :, :1]
    data["static_features"] = cov[:, 0, 1:]
    zero = np.zeros((cov.shape[0], 1, data["prev_treatments"].shape[-1]))
    data["prev_treatments"] = np.concatenate([zero, data["prev_treatments"]], axis=1)
    return data, scaling_params


def make_train(seed=1, num_patients=1000, coeff=2.0, window_size=15, lag=0, seq_length=60,
               treatment_mode="multiclass"):
    """The collection's first subset (dataset.py:589-592): np.random.seed(seed), then the train factual
    cohort.  Returns (processed data, scaling params, raw simulation)."""
    rs = np.random.RandomState(seed)
    p = generate_params(num_patients, coeff, coeff, window_size, lag, rs)
    sim = simulate_factual(p, seq_length, rs)
    data, sp = process_data(sim, get_scaling_params(sim), treatment_mode)
    return data, sp, sim


def de_format_segments(data, sp):
    """The device-side arrays the product's ``SINDY.de_format_segments`` builds (pkpd/utils.py:607-637):
    x [N, T] = prev_outputs[:, 0] ++ unscaled_outputs (unscaled), u [N, U] unscaled statics (patient type; EQ_5 also the t = 0 chemo dosage),
    arm [N, T-1] = argmax(current_treatments), seq_len [N]."""
    std, mean = float(sp["output_stds"]), float(sp["output_means"])
    prev = data["prev_outputs"][..., 0] * std + mean
    x = np.concatenate([prev[:, :1], data["unscaled_outputs"][..., 0]], axis=1)
    U = data["static_features"].shape[-1]
    u = data["static_features"] * sp["inputs_stds"][1:1 + U] + sp["input_means"][1:1 + U]
    arm = np.argmax(data["current_treatments"], axis=-1).astype(np.int64)
    return x, u, arm, data["sequence_lengths"].astype(np.int64)


def simulate_counterfactual_1_step(p, seq_length, rs):
    """cancer_simulation.py:378-563: per patient the factual path and, at every step, the other three
    one-step treatment options.  The assignment window reads the OUTPUT array's row i
    (``cancer_volume[i, ...]``, :449), not the patient's factual series -- restated literally."""
    radio_amt, chemo_amt, half_life = 2.0, 5.0, 1
    window, lag = p["window_size"], p["lag"]
    N = p["initial_stages"].shape[0]
    n_pts = N * seq_length * 4
    V = np.zeros((n_pts, seq_length))
    chemo_a = np.zeros((n_pts, seq_length))
    radio_a = np.zeros((n_pts, seq_length))
    chemo_dose = np.zeros((n_pts, seq_length))
    sl = np.zeros(n_pts)
    ptypes = np.zeros(n_pts)
    idx = 0
    decay = np.exp(-np.log(2) / half_life)
    for i in range(N):
        noise = 0.01 * rs.randn(seq_length)
        recovery_rvs = rs.rand(seq_length)
        fV = np.zeros(seq_length)
        fchemo_d = np.zeros(seq_length)
        fradio_d = np.zeros(seq_length)
        fchemo_a = np.zeros(seq_length)
        fradio_a = np.zeros(seq_length)
        chemo_rvs = rs.rand(seq_length)
        radio_rvs = rs.rand(seq_length)
        fV[0] = p["initial_volumes"][i]
        alpha, beta, beta_c, rho, K = p["alpha"][i], p["beta"][i], p["beta_c"][i], p["rho"][i], p["K"][i]
        for t in range(0, seq_length - 1):
            cur_chemo = 0.0
            prev_chemo = 0.0 if t == 0 else fchemo_d[t - 1]
            used = V[i, max(t - window - lag, 0):max(t - lag + 1, 0)] if t >= lag else np.zeros((1,))
            chemo_prob, radio_prob = _assign_prob(p, i, used)
            if radio_rvs[t] < radio_prob:
                fradio_a[t] = 1
                fradio_d[t] = radio_amt
            if chemo_rvs[t] < chemo_prob:
                fchemo_a[t] = 1
                cur_chemo = chemo_amt
            fchemo_d[t] = prev_chemo * decay + cur_chemo
            fV[t + 1] = fV[t] * (1 + rho * np.log(K / fV[t]) - beta_c * fchemo_d[t]
                                 - (alpha * fradio_d[t] + beta * fradio_d[t] ** 2) + noise[t + 1])
            fV[t + 1] = np.clip(fV[t + 1], 0, TUMOUR_DEATH_THRESHOLD)
            V[idx] = fV
            chemo_a[idx] = fchemo_a
            radio_a[idx] = fradio_a
            chemo_dose[idx] = fchemo_d
            ptypes[idx] = p["patient_types"][i]
            sl[idx] = int(t) + 1
            idx += 1
            for opt in ((0, 0), (0, 1), (1, 0), (1, 1)):
                if fchemo_a[t] == opt[0] and fradio_a[t] == opt[1]:
                    continue
                c_dose = chemo_amt if opt[0] == 1 else 0.0
                r_dose = radio_amt if opt[1] == 1 else 0.0
                cf_chemo_d = prev_chemo * decay + c_dose
                cf_V = fV[t] * (1 + rho * np.log(K / fV[t]) - beta_c * cf_chemo_d
                                - (alpha * r_dose + beta * r_dose ** 2) + noise[t + 1])
                V[idx][:t + 2] = np.append(fV[:t + 1], [cf_V])
                chemo_a[idx][:t + 1] = np.append(fchemo_a[:t], [opt[0]])
                radio_a[idx][:t + 1] = np.append(fradio_a[:t], [opt[1]])
                chemo_dose[idx][:t + 1] = np.append(fchemo_d[:t], [cf_chemo_d])
                ptypes[idx] = p["patient_types"][i]
                sl[idx] = int(t) + 1
                idx += 1
            if fV[t + 1] >= TUMOUR_DEATH_THRESHOLD or recovery_rvs[t] <= np.exp(-fV[t + 1] * TUMOUR_CELL_DENSITY):
                break
    V = _observation_noise(V, p, rs)[:idx]          # drawn over the whole preallocated array
    return {"cancer_volume": V, "chemo_application": chemo_a[:idx], "radio_application": radio_a[:idx],
            "chemo_dosage": chemo_dose[:idx], "sequence_lengths": sl[:idx], "patient_types": ptypes[:idx]}


def simulate_counterfactuals_treatment_seq(p, seq_length, projection_horizon, rs, cf_seq_mode="sliding_treatment"):
    """cancer_simulation.py:566-773 (sliding_treatment: one chemo or one radio dose at each of the tau
    future steps); the assignment window reads the output array's row i (:652), as in the one-step set."""
    tau = projection_horizon
    if cf_seq_mode != "sliding_treatment":
        raise NotImplementedError(cf_seq_mode)
    chemo_arr = np.stack([np.eye(tau, dtype=int), np.zeros((tau, tau), dtype=int)], axis=-1)
    radio_arr = np.stack([np.zeros((tau, tau), dtype=int), np.eye(tau, dtype=int)], axis=-1)
    options = np.concatenate([chemo_arr, radio_arr])
    radio_amt, chemo_amt, half_life = 2.0, 5.0, 1
    window, lag = p["window_size"], p["lag"]
    N = p["initial_stages"].shape[0]
    n_pts = len(options) * N * seq_length
    V = np.zeros((n_pts, seq_length + tau))
    chemo_a = np.zeros((n_pts, seq_length + tau))
    radio_a = np.zeros((n_pts, seq_length + tau))
    chemo_dose = np.zeros((n_pts, seq_length + tau))
    sl = np.zeros(n_pts)
    ptypes = np.zeros(n_pts)
    pids = np.zeros(n_pts)
    pcur = np.zeros(n_pts)
    idx = 0
    decay = np.exp(-np.log(2) / half_life)
    for i in range(N):
        noise = 0.01 * rs.randn(seq_length + tau)
        recovery_rvs = rs.rand(seq_length)
        fV = np.zeros(seq_length)
        fchemo_d = np.zeros(seq_length)
        fradio_d = np.zeros(seq_length)
        fchemo_a = np.zeros(seq_length)
        fradio_a = np.zeros(seq_length)
        chemo_rvs = rs.rand(seq_length)
        radio_rvs = rs.rand(seq_length)
        fV[0] = p["initial_volumes"][i]
        alpha, beta, beta_c, rho, K = p["alpha"][i], p["beta"][i], p["beta_c"][i], p["rho"][i], p["K"][i]
        for t in range(0, seq_length - 1):
            cur_chemo = 0.0
            prev_chemo = 0.0 if t == 0 else fchemo_d[t - 1]
            used = V[i, max(t - window - lag, 0):max(t - lag + 1, 0)] if t >= lag else np.zeros((1,))
            chemo_prob, radio_prob = _assign_prob(p, i, used)
            if radio_rvs[t] < radio_prob:
                fradio_a[t] = 1
                fradio_d[t] = radio_amt
            if chemo_rvs[t] < chemo_prob:
                fchemo_a[t] = 1
                cur_chemo = chemo_amt
            fchemo_d[t] = prev_chemo * decay + cur_chemo
            fV[t + 1] = fV[t] * (1 + rho * np.log(K / fV[t]) - beta_c * fchemo_d[t]
                                 - (alpha * fradio_d[t] + beta * fradio_d[t] ** 2) + noise[t + 1])
            fV[t + 1] = np.clip(fV[t + 1], 0, TUMOUR_DEATH_THRESHOLD)
            for opt in options:
                cV = np.zeros(t + 1 + tau + 1)
                cchemo_a = np.zeros(t + 1 + tau)
                cradio_a = np.zeros(t + 1 + tau)
                cchemo_d = np.zeros(t + 1 + tau)
                cradio_d = np.zeros(t + 1 + tau)
                cV[:t + 2] = fV[:t + 2]
                cchemo_a[:t + 1] = fchemo_a[:t + 1]
                cradio_a[:t + 1] = fradio_a[:t + 1]
                cchemo_d[:t + 1] = fchemo_d[:t + 1]
                cradio_d[:t + 1] = fradio_d[:t + 1]
                for pt in range(tau):
                    ct = t + 1 + pt
                    prev_d = cchemo_d[ct - 1]
                    c_dose = 0.0
                    cradio_d[ct] = 0.0
                    if opt[pt][0] == 1:
                        cchemo_a[ct] = 1
                        c_dose = chemo_amt
                    if opt[pt][1] == 1:
                        cradio_a[ct] = 1
                        cradio_d[ct] = radio_amt
                    cchemo_d[ct] = prev_d * decay + c_dose
                    cV[ct + 1] = cV[ct] * (1 + rho * np.log(K / (cV[ct] + 1e-07) + 1e-07) - beta_c * cchemo_d[ct]
                                           - (alpha * cradio_d[ct] + beta * cradio_d[ct] ** 2) + noise[ct + 1])
                if np.isnan(cV).any():
                    continue
                V[idx][:t + 1 + tau + 1] = cV
                chemo_a[idx][:t + 1 + tau] = cchemo_a
                radio_a[idx][:t + 1 + tau] = cradio_a
                chemo_dose[idx][:t + 1 + tau] = cchemo_d
                ptypes[idx] = p["patient_types"][i]
                pids[idx] = i
                pcur[idx] = t
                sl[idx] = int(t) + tau + 1
                idx += 1
            if fV[t + 1] >= TUMOUR_DEATH_THRESHOLD or recovery_rvs[t] <= np.exp(-fV[t + 1] * TUMOUR_CELL_DENSITY):
                break
    V = _observation_noise(V, p, rs)[:idx]          # drawn over the whole preallocated array
    return {"cancer_volume": V, "chemo_application": chemo_a[:idx], "radio_application": radio_a[:idx],
            "chemo_dosage": chemo_dose[:idx], "sequence_lengths": sl[:idx], "patient_types": ptypes[:idx],
            "patient_ids_all_trajectories": pids[:idx],
            "patient_current_t": pcur[:idx]}


def make_collection(seed=1, num_patients=None, coeff=2.0, window_size=15, lag=0, seq_length=60, projection_horizon=5,
                    treatment_mode="multiclass", with_tests=True, equation=None):
    """SyntheticCancerDatasetCollection (dataset.py:556-605) + process_data_multi (dataset_collection.py:74-86):
    one np.random.seed(seed) stream for train / val (factual), test one-step and test tau-step
    counterfactual subsets; every subset scaled with the train statistics; the tau-step set's
    ``data_processed_seq`` holds the last-tau targets (process_sequential_test).  ``equation``
    "EQ_5_A".."EQ_5_D": SyntheticContinuousDatasetCollection (continuous/dataset.py:565-618), whose every
    subset re-seeds np.random.seed(seed) (:51).  Returns a dict of ``insite_ref.Subset`` with norm_const =
    TUMOUR_DEATH_THRESHOLD."""
    from . import insite_ref as R
    num_patients = num_patients or {"train": 1000, "val": 100, "test": 100}
    rs = np.random.RandomState(seed)

    def stream():
        return np.random.RandomState(seed) if equation is not None else rs

    sims = {}
    r = stream()
    sims["train"] = simulate_factual(generate_params(num_patients["train"], coeff, coeff, window_size, lag, r, equation),
                                     seq_length, r)
    r = stream()
    sims["val"] = simulate_factual(generate_params(num_patients["val"], coeff, coeff, window_size, lag, r, equation),
                                   seq_length, r)
    if with_tests:
        r = stream()
        p = generate_params(num_patients["test"], coeff, coeff, window_size, lag, r, equation)
        sims["test_cf_one_step"] = simulate_counterfactual_1_step(p, seq_length, r)
        r = stream()
        p = generate_params(num_patients["test"], coeff, coeff, window_size, lag, r, equation)
        sims["test_cf_treatment_seq"] = simulate_counterfactuals_treatment_seq(p, seq_length, projection_horizon, r)
    scaling = get_scaling_params(sims["train"])
    out = {}
    for name, sim in sims.items():
        data, sp = process_data(sim, scaling, treatment_mode, equation, include_continuous_treatment=equation is not None)
        seq = R.process_sequential_test(data, sp, projection_horizon) if name == "test_cf_treatment_seq" else None
        out[name] = R.Subset(name, data, sp, seq, TUMOUR_DEATH_THRESHOLD)
    return out


def sindy_pipeline(coll, threshold=1e-3, alpha=0.5, dt=None, fd="order1"):
    """train_sindy.main for the cancer_sim SINDy backbone (segment fits, 4-arm Euler-5 rollout,
    sindy.py:193-216, 289-312, 371-431) with the reference's metrics."""
    from . import insite_ref as R
    from . import segments_ref as S
    dt = R.STANDARD_DT if dt is None else dt
    tr = coll["train"]
    x, u, arm, sl = de_format_segments(tr.data, tr.scaling_params)
    joint, _, _, exps = S.sindy_fit_segments(x, u, arm, sl, dt, threshold, alpha, fd=fd)
    U = u.shape[1]
    names = R.library_names(exps, ["x0"] + [f"u{i}" for i in range(U)])
    res = {"joint_coefs": joint, "exps": exps, "names": names,
           "global_equation_string": S.global_equation_string(joint, names)}

    def predict(sub):
        prev, st = R.unscale_inputs(sub.data, sub.scaling_params, 1, U)
        return R.rollout(prev[:, 0], st, np.argmax(sub.data["current_treatments"], axis=-1), joint, exps, dt, "euler5")

    norm = TUMOUR_DEATH_THRESHOLD
    one = coll.get("test_cf_one_step")
    if one is not None:
        pu = predict(one)
        o, a_, l_ = R.masked_rmse(pu[..., None], one.data["unscaled_outputs"], one.data["active_entries"], norm,
                                  one_step_counterfactual=True)
        res.update(encoder_test_rmse_orig=o, encoder_test_rmse_all=a_, encoder_test_rmse_last=l_)
    seqs = coll.get("test_cf_treatment_seq")
    if seqs is not None:
        pu = predict(seqs)
        tau = seqs.data_processed_seq["outputs"].shape[1]
        sl_ = R.autoregressive_slice(pu[..., None], seqs.data["sequence_lengths"], tau)
        r = R.n_step_rmses(sl_, seqs.data_processed_seq["unscaled_outputs"], seqs.data_processed_seq["active_entries"],
                           norm)
        for k, v in enumerate(r):
            res[f"decoder_test_rmse_{k + 2}-step"] = v
    return res


def joint_pipeline(coll, threshold=1e-3, alpha=0.5, dt=None, fd="order1"):
    """The one-ODE ablation (run.py:198-201: joint_model, multilabel treatments) on cancer_sim: ONE fit
    over X = unscaled_outputs[:seq_len] with library inputs (x0, chemo, radio, patient type)
    (pkpd/utils.py:493-497, 664-672; sindy.py:203), rolled out with the per-step treatments as inputs
    (sindy.py:317-322).  ``coll`` from ``make_collection(treatment_mode="multilabel")``."""
    from . import insite_ref as R
    dt = R.STANDARD_DT if dt is None else dt
    tr = coll["train"]
    _, stat = R.unscale_inputs(tr.data, tr.scaling_params, 1, 1)
    x = tr.data["unscaled_outputs"][..., 0]
    inputs = np.asarray(tr.data["current_treatments"], dtype=np.float64)
    rows = tr.data["sequence_lengths"].astype(np.int64)
    n_in = inputs.shape[-1]
    exps = R.poly_library(1 + n_in + stat.shape[1], 2, True)
    names = R.library_names(exps, ["x0"] + [f"u{i}" for i in range(n_in + stat.shape[1])])
    Z, Y = R.build_regression_joint(x, inputs, stat, rows, dt, fd)
    c, _, _ = R.stlsq(R.eval_library(exps, Z), Y, threshold, alpha)
    res = {"joint_coefs": c[None, :], "exps": exps,
           "global_equation_string": f"Joint Model: x_dot = {R.equation_terms(c, names)}"}

    def predict(sub):
        prev, st = R.unscale_inputs(sub.data, sub.scaling_params, 1, 1)
        return R.rollout_inputs(prev[:, 0], st, np.asarray(sub.data["current_treatments"], dtype=np.float64), c, exps,
                                dt, "euler5")

    norm = TUMOUR_DEATH_THRESHOLD
    one = coll.get("test_cf_one_step")
    if one is not None:
        pu = predict(one)
        o, a_, l_ = R.masked_rmse(pu[..., None], one.data["unscaled_outputs"], one.data["active_entries"], norm,
                                  one_step_counterfactual=True)
        res.update(encoder_test_rmse_orig=o, encoder_test_rmse_all=a_, encoder_test_rmse_last=l_)
    seqs = coll.get("test_cf_treatment_seq")
    if seqs is not None:
        pu = predict(seqs)
        tau = seqs.data_processed_seq["outputs"].shape[1]
        sl_ = R.autoregressive_slice(pu[..., None], seqs.data["sequence_lengths"], tau)
        r = R.n_step_rmses(sl_, seqs.data_processed_seq["unscaled_outputs"], seqs.data_processed_seq["active_entries"],
                           norm)
        for k, v in enumerate(r):
            res[f"decoder_test_rmse_{k + 2}-step"] = v
    return res
