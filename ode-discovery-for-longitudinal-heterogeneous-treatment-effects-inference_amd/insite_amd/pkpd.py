"""PK/PD dataset collection (input side of the hot path: SURVEY.md §8 A11, F1, F3).

Drop-in for the reference's ``SyntheticPkpdDatasetCollection`` / ``SyntheticPkpdDataset``
(``libs_m/ct/src/data/pkpd/dataset.py:18-192, 395-475, 535-607``) and the simulators of
``libs_m/ct/src/data/pkpd/pkpd_simulation.py`` (``get_standard_params`` :96-203,
``simulate_factual`` :205-309, ``simulate_counterfactual_1_step`` :341-471,
``simulate_counterfactuals_treatment_seq`` :474-667, ``get_scaling_params`` :670-693).

Cohorts are generated with torch on the requested device (the MI355X by default) and handed to
the model in the reference's layout: ``dataset.data`` is a dict of numpy arrays
(``prev_outputs [N,T-1,1]``, ``current_treatments [N,T-1,2]`` one-hot, ``static_features [N,2]``,
``outputs``/``unscaled_outputs``/``active_entries [N,T-1,1]``, ``sequence_lengths [N]``, ...),
``dataset.scaling_params`` and ``dataset.norm_const = 50``.

Random draws (``rng=``):

* ``"threefry"`` (default): the reference's own key schedule and draws -- ``PRNGKey(seed)`` per
  subset, ``key, subkey = split(key)`` before every draw, jax's uniform / normal / permutation /
  choice transforms -- with the Threefry-2x32 words produced on the device by
  ``insite_threefry2x32_iota_u32`` (insite_amd/threefry.py).  The reference's cohorts are
  reproduced (tests/test_gpu_threefry.py), so ``run.py`` reproduces its logged rows.  Needs the
  HIP library and a GPU device.
* ``"torch"``: torch's generator with the same distributions and time grids, seeded per
  (seed, subset); host-side tests on CPU tensors.

The time grids are the reference's: ``arange(0, 10, dt)`` for the factual and one-step
simulators, ``arange(T + 1) * dt`` with accumulated ``+ dt`` windows for the tau-step one, each
interval integrated by 5 Euler sub-steps of ``(t1 - t0) / 5`` (utils.py:68-94).
"""
from __future__ import annotations

import numpy as np
import torch

MAX_VALUE = 50.0                 # pkpd/utils.py:37
STEPS_FOR_DT = 5                 # pkpd/utils.py:40
MAX_TIME_HORIZON = 10.0          # pkpd/utils.py:48
OBSERVATION_NOISE = 0.01         # pkpd_simulation.py:44
RECOVERY_MULTIPLIER = 5.8e11     # pkpd_simulation.py:46
EQUATIONS = ("EQ_4_A", "EQ_4_B", "EQ_4_C", "EQ_4_D", "EQ_4_M")
_SUBSET_STREAM = {"train": 0, "val": 1, "test_cf_one_step": 2, "test_cf_treatment_seq": 3}


def _noisy(equation: str) -> bool:
    return equation.split("_")[-1] in ("B", "C", "D")


class _TorchRng:
    """torch's generator on ``device``, one per (seed, subset); same interface as ``_ThreefryRng``
    (the key-schedule hooks are no-ops)."""

    def __init__(self, seed: int, subset: str, device):
        self.dev = torch.device(device)
        self.g = torch.Generator(device=self.dev)
        self.g.manual_seed(int(seed) * 7919 + 104729 * _SUBSET_STREAM[subset] + 17)

    def normal(self, *shape):
        return torch.randn(shape, generator=self.g, device=self.dev, dtype=torch.float64)

    def uniform(self, *shape, lo: float = 0.0, hi: float = 1.0):
        u = torch.rand(shape, generator=self.g, device=self.dev, dtype=torch.float64)
        return u if (lo, hi) == (0.0, 1.0) else u * (hi - lo) + lo

    def permutation(self, n: int):
        return torch.randperm(int(n), generator=self.g, device=self.dev)

    def choice2(self, n: int, values):
        return torch.where(self.uniform(n) < 0.5, values[0], values[1])

    def skip(self):
        pass

    def split_first(self, num: int):
        pass


class _ThreefryRng:
    """The reference's jax.random key threading for one key (``key, subkey = split(key)`` before
    every draw), words from the device Threefry kernel (insite_amd/threefry.py)."""

    def __init__(self, key, device):
        from . import threefry
        self._tf = threefry
        self.s = threefry.Stream(key, device)
        self.dev = self.s.dev

    def normal(self, *shape):
        return self.s.normal(*shape)

    def uniform(self, *shape, lo: float = 0.0, hi: float = 1.0):
        return self.s.uniform(*shape, lo=lo, hi=hi)

    def permutation(self, n: int):
        return self.s.permutation(n)

    def choice2(self, n: int, values):
        """``jax.random.choice(key, [v0, v1], (n,))`` = ``a[randint(key, (n,), 0, 2)]``; randint over a
        span of 2 with 64-bit draws (multiplier 2^32 mod 2 = 0) keeps ``lower_bits mod 2`` of the second
        split subkey's bits (jax 0.4.x random.py ``_randint``).  Parity unpinned: no logged EQ_4_M run."""
        sub = self.s._sub()
        _, k2 = self._tf.split(sub, 2, self.dev)
        lower = self._tf.random_bits(k2, 64, (int(n),), self.dev)
        return torch.where((lower & 1) == 0, values[0], values[1])

    def skip(self):
        """A ``key, subkey = split(key)`` whose draw the simulator never reads (recovery rvs)."""
        self.s._sub()

    def split_first(self, num: int):
        self.s.split_first(num)


def subset_rngs(kind: str, seed: int, subset: str, device):
    """(params rng, simulator rng) for one subset.  threefry: ``key = PRNGKey(seed)``, then
    ``key, k_params = split(key)``; ``key, k_sim = split(key)`` (pkpd/dataset.py:52-54, 64-71) -- every
    subset restarts from the same seed, as the reference does (dataset.py:594-603)."""
    if kind == "threefry":
        dev = torch.device(device)
        if dev.type != "cuda":
            raise RuntimeError("rng='threefry' draws on the device (HIP kernel); pass a cuda device "
                               "(rng='torch' is the host-side generator)")
        from . import threefry
        kp, ks = threefry.subset_streams(seed, dev)
        return _ThreefryRng(kp.key, dev), _ThreefryRng(ks.key, dev)
    if kind == "torch":
        r = _TorchRng(seed, subset, device)
        return r, r
    raise ValueError(f"rng {kind!r}: 'threefry' or 'torch'")


def draw_params(n: int, equation: str, rng) -> dict:
    """Patient parameters (get_standard_params, pkpd_simulation.py:96-203)."""
    if equation not in EQUATIONS:
        raise NotImplementedError(f"equation {equation!r} (PK/PD EQ_4 family only)")
    scale = 0.5
    c_0 = rng.normal(n) * (0.1 * scale) + scale                       # :117-118
    c_1 = rng.normal(n) * (0.1 * scale) + scale                       # :121-122
    C_0, C_1 = c_0.clone(), c_1.clone()                               # EQ_4_A / B
    if equation in ("EQ_4_C", "EQ_4_D"):                              # :128-150
        C_0 = c_0 + 0.1 * scale
        C_1 = c_1 + 0.3 * scale
        if equation == "EQ_4_D":                                      # :152-158, one shift per arm
            C_0 = rng.normal() * (0.5 * scale) + C_0
            C_1 = rng.normal() * (0.5 * scale) + C_1
    elif equation == "EQ_4_M":                                        # :159-165 bimodal
        C_0 = c_0 + rng.choice2(n, (0.1 * scale, 0.3 * scale))
        C_1 = c_1 + rng.choice2(n, (0.1 * scale, 0.3 * scale))
    x0 = rng.uniform(n, lo=1.0, hi=MAX_VALUE)                         # :181-182
    perm = rng.permutation(n)                                         # :195-201
    return {"initial_volumes": x0[perm], "hidden_C_0": C_0[perm], "hidden_C_1": C_1[perm],
            "observed_static_c_0": c_0[perm], "observed_static_c_1": c_1[perm]}


def _assign(x0, rv, conf_coeff):
    """``rv < 1 / (1 + exp(-gamma (x0 - 25)))``, gamma = coeff / 50 (pkpd_simulation.py:76-94, 255-259)."""
    gamma = conf_coeff / MAX_VALUE
    prob = 1.0 / (1.0 + torch.exp(-gamma * (x0 - MAX_VALUE / 2.0)))
    return (rv < prob).to(torch.int64)


def _interval(v, C, t0: float, t1: float):
    """``odeint(dy_dt, v, [t0, t1])[1]`` of dy/dt = -C y: HMAX < t1 - t0, so 5 Euler sub-steps of
    (t1 - t0) / 5 (utils.py:68-94; pkpd_simulation.py:69-73)."""
    h = (t1 - t0) / STEPS_FOR_DT
    for _ in range(STEPS_FOR_DT):
        v = v + (-C * v) * h
    return v


def _first_true(mask):
    """(any, first index) along the last axis."""
    anyv = mask.any(dim=-1)
    first = torch.argmax(mask.to(torch.int8), dim=-1)
    return anyv, first


def simulate_factual(p: dict, T: int, rng, equation: str, conf_coeff: float) -> dict:
    """Factual cohort (pkpd_simulation.py:205-309)."""
    t_grid = np.arange(0, MAX_TIME_HORIZON, MAX_TIME_HORIZON / T)     # :261
    x0 = p["initial_volumes"]
    n = x0.numel()
    rec_rv = rng.uniform(n, T)                                        # :233-234
    a = _assign(x0, rng.uniform(n), conf_coeff)                       # :235-236, 255-259
    C = torch.where(a == 0, p["hidden_C_0"], p["hidden_C_1"])
    V = torch.empty((n, T), dtype=torch.float64, device=x0.device)
    V[:, 0] = x0
    for k in range(1, T):                                             # :262
        V[:, k] = _interval(V[:, k - 1], C, float(t_grid[k - 1]), float(t_grid[k]))
    seq = torch.full((n,), T - 1, dtype=torch.int64, device=x0.device)  # :254
    t = torch.arange(T, device=x0.device)[None, :]
    rec_any, rec_first = _first_true(rec_rv < torch.exp(-V * RECOVERY_MULTIPLIER))   # :264-265
    V = torch.where(rec_any[:, None] & (t >= rec_first[:, None]), 0.0, V)
    seq = torch.where(rec_any, rec_first + 1, seq)
    dead_any, dead_first = _first_true(V > MAX_VALUE)                                 # :267-268
    V = torch.where(dead_any[:, None] & (t >= dead_first[:, None]), MAX_VALUE, V)
    seq = torch.where(dead_any, dead_first + 1, seq)
    if _noisy(equation):                                              # :289-291
        V = V + OBSERVATION_NOISE * rng.normal(n, T)
    treat = torch.zeros((n, T), dtype=torch.float64, device=x0.device)
    treat[:, : T - 1] = a[:, None].to(torch.float64)                 # :270, :296
    return {"cancer_volume": V, "treatment_application": treat, "sequence_lengths": seq.to(torch.float64),
            "observed_static_c_0": p["observed_static_c_0"], "observed_static_c_1": p["observed_static_c_1"]}


def simulate_counterfactual_1_step(p: dict, T: int, rng, equation: str, conf_coeff: float) -> dict:
    """Every one-step-ahead counterfactual (pkpd_simulation.py:341-471): per patient and step i,
    a factual row and a row whose treatment flips at step i; 2(T-1) rows per patient."""
    t_grid = np.arange(0, MAX_TIME_HORIZON, MAX_TIME_HORIZON / T)     # :394-395
    x0 = p["initial_volumes"]
    n, dev = x0.numel(), x0.device
    rng.skip()                                                        # recovery rvs (:380-381), unused
    a = _assign(x0, rng.uniform(n), conf_coeff)                       # :382-383
    C = torch.where(a == 0, p["hidden_C_0"], p["hidden_C_1"])
    Ccf = torch.where(a == 0, p["hidden_C_1"], p["hidden_C_0"])
    V = torch.empty((n, T), dtype=torch.float64, device=dev)
    V[:, 0] = x0
    cf = torch.empty((n, T - 1), dtype=torch.float64, device=dev)
    for k in range(T - 1):                                            # :344-350
        t0, t1 = float(t_grid[k]), float(t_grid[k + 1])
        cf[:, k] = _interval(V[:, k], Ccf, t0, t1)
        V[:, k + 1] = _interval(V[:, k], C, t0, t1)
    i = torch.arange(T - 1, device=dev)[:, None]                      # row pair index
    t = torch.arange(T, device=dev)[None, :]
    fact = torch.where(t < i + 2, V[:, None, :], 0.0)                 # [n, T-1, T]
    cfr = torch.where(t < i + 1, V[:, None, :], 0.0) + torch.where(t == i + 1, cf[:, :, None], 0.0)
    vol = torch.stack([fact, cfr], dim=2).reshape(n, 2 * (T - 1), T)  # rows 2i, 2i+1 (:405-413)
    tt = torch.arange(T - 1, device=dev)[None, :]
    af = a[:, None, None].to(torch.float64)
    trt_f = torch.where(tt < i + 1, af, 0.0)
    trt_c = torch.where(tt < i, af, 0.0) + torch.where(tt == i, 1.0 - af, 0.0)
    trt = torch.stack([trt_f, trt_c], dim=2).reshape(n, 2 * (T - 1), T - 1)
    sl = (torch.arange(T - 1, device=dev) + 1).repeat_interleave(2)[None, :].expand(n, -1)
    if _noisy(equation):                                              # :438-444
        vol = vol + OBSERVATION_NOISE * rng.normal(*vol.shape)
    rows = n * 2 * (T - 1)
    treat = torch.zeros((rows, T), dtype=torch.float64, device=dev)
    treat[:, : T - 1] = trt.reshape(rows, T - 1)
    reps = 2 * (T - 1)
    return {"cancer_volume": vol.reshape(rows, T), "treatment_application": treat,
            "sequence_lengths": sl.reshape(rows).to(torch.float64),
            "observed_static_c_0": p["observed_static_c_0"].repeat_interleave(reps),
            "observed_static_c_1": p["observed_static_c_1"].repeat_interleave(reps)}


def simulate_counterfactuals_treatment_seq(p: dict, T: int, tau: int, rng, equation: str,
                                           conf_coeff: float) -> dict:
    """tau-step sliding-treatment counterfactuals (pkpd_simulation.py:474-487, 516-667): per
    patient and step i, 2*tau treatment plans (one-hot and inverted one-hot over tau steps)."""
    dt = MAX_TIME_HORIZON / T
    t_grid = np.arange(0, T + 1).astype(np.float64) * dt              # :537
    x0 = p["initial_volumes"]
    n, dev = x0.numel(), x0.device
    rng.skip()                                                        # recovery rvs (:555-556), unused
    a = _assign(x0, rng.uniform(n), conf_coeff)                       # :557-558
    C0, C1 = p["hidden_C_0"], p["hidden_C_1"]
    C = torch.where(a == 0, C0, C1)
    eye = torch.eye(tau, dtype=torch.int64, device=dev)
    plans = torch.cat([eye, 1 - eye], dim=0)                          # [2tau, tau] (:476-489)
    V = torch.empty((n, T + 1), dtype=torch.float64, device=dev)
    V[:, 0] = x0
    V[:, 1] = _interval(x0, C, float(t_grid[0]), float(t_grid[1]))   # :574
    P = 2 * tau
    cfv = torch.empty((n, T - 1, P, tau), dtype=torch.float64, device=dev)
    Cp = torch.where(plans[None] == 0, C0[:, None, None], C1[:, None, None])   # [n, P, tau]
    for i in range(T - 1):                                            # t_tuples (t[i+1], t[i+2]) :571-600
        ts, te = float(t_grid[i + 1]), float(t_grid[i + 2])
        v = V[:, i + 1][:, None].expand(n, P)
        for j in range(tau):                                          # windows advance by += dt (:478-486)
            v = _interval(v, Cp[:, :, j], ts, te)
            ts, te = ts + dt, te + dt
            cfv[:, i, :, j] = v
        V[:, i + 2] = _interval(V[:, i + 1], C, float(t_grid[i + 1]), float(t_grid[i + 2]))   # :513
    L = T + tau
    i = torch.arange(T - 1, device=dev)[:, None, None]                # [T-1, 1, 1]
    t = torch.arange(L, device=dev)[None, None, :]                    # [1, 1, L]
    Vp = torch.cat([V, torch.zeros((n, L - (T + 1)), dtype=torch.float64, device=dev)], dim=1)
    hist = torch.where(t < i + 2, Vp[:, None, None, :], 0.0)          # [n, T-1, 1, L]
    j = t - (i + 2)                                                   # position inside the cf window
    inwin = (j >= 0) & (j < tau)
    jc = j.clamp(0, tau - 1).expand(T - 1, P, L)
    cfw = torch.gather(cfv, 3, jc[None].expand(n, -1, -1, -1))        # [n, T-1, P, L]
    vol = hist + torch.where(inwin, cfw, 0.0)                         # :608-613
    tt = torch.arange(L - 1, device=dev)[None, None, :]
    af = a[:, None, None, None].to(torch.float64)
    jt = tt - (i + 1)
    inw_t = (jt >= 0) & (jt < tau)
    plan_v = torch.gather(plans[None].expand(T - 1, -1, -1).to(torch.float64), 2,
                          jt.clamp(0, tau - 1).expand(T - 1, P, L - 1))
    trt = torch.where(tt < i + 1, af, 0.0) + torch.where(inw_t, plan_v, 0.0)[None]
    nr = (T - 1) * P
    sl = (torch.arange(T - 1, device=dev) + 1 + tau).repeat_interleave(P)[None, :].expand(n, -1)
    rng.split_first(n + 1)                                            # :616 key, *subkeys = split(key, n + 1)
    if _noisy(equation):                                              # :639-646
        vol = vol + OBSERVATION_NOISE * rng.normal(*vol.shape)
    rows = n * nr
    treat = torch.zeros((rows, L), dtype=torch.float64, device=dev)
    treat[:, : L - 1] = trt.reshape(rows, L - 1)
    return {"cancer_volume": vol.reshape(rows, L), "treatment_application": treat,
            "sequence_lengths": sl.reshape(rows).to(torch.float64),
            "observed_static_c_0": p["observed_static_c_0"].repeat_interleave(nr),
            "observed_static_c_1": p["observed_static_c_1"].repeat_interleave(nr)}


def get_scaling_params(sim: dict):
    """Mean / population std over active entries (pkpd_simulation.py:670-693)."""
    V = sim["cancer_volume"]
    seq = sim["sequence_lengths"].to(torch.int64)
    act = torch.arange(V.shape[1], device=V.device)[None, :] < seq[:, None]
    vals = V[act]
    mean = {"cancer_volume": float(vals.mean()), "observed_static_c_0": float(sim["observed_static_c_0"].mean()),
            "observed_static_c_1": float(sim["observed_static_c_1"].mean())}
    std = {"cancer_volume": float(vals.std(unbiased=False)),
           "observed_static_c_0": float(sim["observed_static_c_0"].std(unbiased=False)),
           "observed_static_c_1": float(sim["observed_static_c_1"].std(unbiased=False))}
    return mean, std


def process_data(sim: dict, scaling) -> tuple[dict, dict]:
    """Model-facing layout of ``SyntheticPkpdDataset.process_data`` (pkpd/dataset.py:96-192),
    multiclass treatments.  Returns (numpy data dict, scaling_params)."""
    mean, std = scaling
    V = (sim["cancer_volume"] - mean["cancer_volume"]) / std["cancer_volume"]
    c0 = (sim["observed_static_c_0"] - mean["observed_static_c_0"]) / std["observed_static_c_0"]
    c1 = (sim["observed_static_c_1"] - mean["observed_static_c_1"]) / std["observed_static_c_1"]
    app = sim["treatment_application"][:, :-1]                        # :132-133
    onehot = torch.stack([(app == 0), (app == 1)], dim=-1).to(torch.float64)
    n, Tm1 = V.shape[0], V.shape[1] - 1
    cur_cov = torch.stack([V[:, :-1], c0[:, None].expand(n, Tm1), c1[:, None].expand(n, Tm1)], dim=-1)
    outputs = V[:, 1:, None]
    seq = sim["sequence_lengths"].to(torch.int64)
    active = (torch.arange(Tm1, device=V.device)[None, :, None] < seq[:, None, None]).to(torch.float64)
    d = {k: v.cpu().numpy() for k, v in sim.items()}
    d.update({
        "current_treatments": onehot.cpu().numpy(),
        "prev_treatments": torch.cat([torch.zeros((n, 1, 2), dtype=torch.float64, device=V.device), onehot[:, :-1]],
                                     dim=1).cpu().numpy(),
        "current_covariates": cur_cov.cpu().numpy(),
        "outputs": outputs.cpu().numpy(),
        "active_entries": active.cpu().numpy(),
        "unscaled_outputs": (outputs * std["cancer_volume"] + mean["cancer_volume"]).cpu().numpy(),
        "prev_outputs": cur_cov[:, :, :1].cpu().numpy(),
        "static_features": cur_cov[:, 0, 1:].cpu().numpy(),
    })
    sp = {"input_means": np.array([mean["cancer_volume"], mean["observed_static_c_0"], mean["observed_static_c_1"], 0.0]),
          "inputs_stds": np.array([std["cancer_volume"], std["observed_static_c_0"], std["observed_static_c_1"], 1.0]),
          "output_means": mean["cancer_volume"], "output_stds": std["cancer_volume"]}
    return d, sp


def process_sequential_test(data: dict, scaling_params: dict, projection_horizon: int) -> dict:
    """Targets of ``process_sequential_test`` (pkpd/dataset.py:395-475): the last tau outputs of
    every row (tau = projection_horizon)."""
    tau = int(projection_horizon)
    seq = data["sequence_lengths"].astype(np.int64)
    idx = (seq - tau)[:, None] + np.arange(tau)[None, :]
    out = np.take_along_axis(data["outputs"][..., 0], idx, axis=1)[..., None]
    return {"outputs": out, "active_entries": np.ones_like(out),
            "unscaled_outputs": out * scaling_params["output_stds"] + scaling_params["output_means"],
            "sequence_lengths": seq.astype(np.float64)}


class SyntheticPkpdDataset:
    """One subset: ``subset_name``, ``data`` (numpy dict), ``scaling_params``, ``norm_const``,
    and for the tau-step test set ``data_processed_seq`` (pkpd/dataset.py:18-192)."""

    def __init__(self, subset_name: str, sim: dict):
        self.subset_name = subset_name
        self.sim = sim
        self.data = None
        self.scaling_params = None
        self.data_processed_seq = None
        self.norm_const = MAX_VALUE
        self.processed = False

    def get_scaling_params(self):
        return get_scaling_params(self.sim)

    def process_data(self, scaling):
        if not self.processed:
            self.data, self.scaling_params = process_data(self.sim, scaling)
            self.processed = True
        return self.data

    def __len__(self):
        return 0 if self.data is None else len(self.data["sequence_lengths"])


class SyntheticPkpdDatasetCollection:
    """``train_f``, ``val_f``, ``test_cf_one_step``, ``test_cf_treatment_seq``
    (pkpd/dataset.py:557-607).  ``process_data_multi()`` applies the train scaling to every subset
    and builds the tau-step targets (dataset_collection.py:74-86)."""

    def __init__(self, conf_coeff: float, num_patients: dict, equation_str: str, seed: int,
                 max_seq_length: int = 60, projection_horizon: int = 5, device=None, rng: str = "threefry",
                 **kwargs):
        dev = torch.device(device) if device is not None else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        T = int(max_seq_length)
        self.seed = seed
        self.equation = equation_str
        self.projection_horizon = int(projection_horizon)
        self.autoregressive = True
        self.has_vitals = False
        self.processed_data_multi = False
        self.rng = rng
        subsets = {}
        for name, n in (("train", num_patients["train"]), ("val", num_patients["val"])):
            rp, rs = subset_rngs(rng, seed, name, dev)
            subsets[name] = simulate_factual(draw_params(int(n), equation_str, rp), T, rs, equation_str, conf_coeff)
        rp, rs = subset_rngs(rng, seed, "test_cf_one_step", dev)
        one = simulate_counterfactual_1_step(draw_params(int(num_patients["test"]), equation_str, rp), T, rs,
                                             equation_str, conf_coeff)
        rp, rs = subset_rngs(rng, seed, "test_cf_treatment_seq", dev)
        seqs = simulate_counterfactuals_treatment_seq(draw_params(int(num_patients["test"]), equation_str, rp), T,
                                                      self.projection_horizon, rs, equation_str, conf_coeff)
        self.train_f = SyntheticPkpdDataset("train", subsets["train"])
        self.val_f = SyntheticPkpdDataset("val", subsets["val"])
        self.test_cf_one_step = SyntheticPkpdDataset("test", one)
        self.test_cf_treatment_seq = SyntheticPkpdDataset("test", seqs)
        self.train_scaling_params = self.train_f.get_scaling_params()

    def process_data_multi(self):
        if self.processed_data_multi:
            return
        for ds in (self.train_f, self.val_f, self.test_cf_one_step, self.test_cf_treatment_seq):
            ds.process_data(self.train_scaling_params)
        s = self.test_cf_treatment_seq
        s.data_processed_seq = process_sequential_test(s.data, s.scaling_params, self.projection_horizon)
        self.processed_data_multi = True


def dataset_collection(equation: str, num_patients: dict, seed: int, conf_coeff: float = 2.0,
                       max_seq_length: int = 60, projection_horizon: int = 5, device=None, rng: str = "threefry"):
    """Build and process a collection in one call (``get_dataset`` + ``process_data_multi``)."""
    c = SyntheticPkpdDatasetCollection(conf_coeff, num_patients, equation, seed, max_seq_length, projection_horizon,
                                       device=device, rng=rng)
    c.process_data_multi()
    return c

