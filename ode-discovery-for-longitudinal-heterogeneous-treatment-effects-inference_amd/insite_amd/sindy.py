"""The ``+backbone=sindy`` plugin on MI355X: drop-in for the reference ``SINDY`` model
(``libs_m/ct/src/models/sindy.py:57-431, 717-760``; metrics inherited from
``libs_m/ct/src/models/time_varying_model.py:236-313``).

Same constructor (``SINDY(args, dataset_collection)``), methods (``fit``, ``get_predictions``,
``get_autoregressive_predictions``, ``get_normalised_masked_rmse``,
``get_normalised_n_step_rmses``), attributes (``global_equation_string``, ``joint_coefs``,
``feature_library_names``, ``insite``, ``hparams``) and error behaviour (Python exceptions;
``AssertionError`` on NaN predictions).  The two inner call sites of the reference run on the GPU
through the C ABI (include/insite_hip.h):

* ``SINDy(...).fit(X_a, u=U_a, t=dt, multiple_trajectories=True)`` per arm (sindy.py:190-192)
  -> ``insite_sindy_fit_f64``: smoothing + 4th-order FD + library + per-arm Gram in one streaming
  kernel, then the reduction fused with STLSQ + unbias for every arm.
* ``jit(vmap(simulate_cancer_volume))`` (sindy.py:413-431) -> ``insite_rollout_f64`` (Euler-5).
* ``insite: true`` — ``pmap(vmap(simulate_cancer_volume_with_fine_tuning))`` (sindy.py:433-715): the
  per-patient BFGS refinement -> ``insite_refine_f64`` (one lane per patient; 4-arm datasets:
  ``insite_refine_arms_f64``).

The DE-format extraction (A1, pkpd/utils.py:523-606), the tau-step slice (A9) and the masked
squared-error sums of the metrics (A10) also run on the device; only scalars and the returned
prediction arrays cross back to the host.  The cancer_sim / EQ_5 datasets run the
treatment-segment discovery (``insite_sindy_fit_segments_f64``), the 4-arm rollout and, with
``insite: true``, the 4-arm refinement.  The ablations run through the general one-state path
(``insite_gen_gram_f64``): ``ablation_more_complex_basis_functions`` (PolynomialLibrary(degree=4,
interaction_only=False), sindy.py:185-186; EQ_4) and ``joint_model`` (one regression with the multilabel
treatment(s) as library inputs, pkpd/utils.py:486-497, 639-672; sindy.py:283-288, 313-322), whose RHS
is folded per treatment combination into the per-arm rollout; with ``insite: true`` both refine on the
GPU (``insite_refine_general_f64``: the joint model's coefficients act on the treatment combinations their
inputs switch on; the degree-4 library runs the state-polynomial refinement kernels).  The degree-4 library
on the treatment-segment datasets runs ``insite_gen_gram_segments_f64`` (per-arm power moments of the
segment rows).  Not on the MI355X path (raises ``NotImplementedError``): weak SINDy.
"""
from __future__ import annotations

import logging

import numpy as np
import torch

from . import ops
from .library import polynomial_library

logger = logging.getLogger(__name__)

MAX_SEQUENCE_LENGTH = 60
MAX_TIME_HORIZON = 10.0
STANDARD_DT = MAX_TIME_HORIZON / MAX_SEQUENCE_LENGTH   # pkpd/utils.py:53; SINDY.dt (sindy.py:89)
RHS_COEF_EPS = 1e-3                                    # pkpd/utils.py:388


# scipy.signal.savgol_filter(window_length=5, polyorder=3, mode='interp') weights: interior taps and the
# polynomial-fit edge rows (the same table as the HIP kernels' sg_pos*/sg_interior)
_SG53 = np.array([[69, 4, -6, 4, -1], [4, 54, 24, -16, 4], [-3, 12, 17, 12, -3], [4, -16, 24, 54, 4],
                  [-1, 4, -6, 4, 69]], dtype=np.float64) / np.array([70, 70, 35, 70, 70], dtype=np.float64)[:, None]


def savgol_5_3_rows(V: torch.Tensor) -> torch.Tensor:
    """savgol(5, 3, mode='interp') along the time axis of [N, T] device rows (T >= 5)."""
    W = torch.as_tensor(_SG53, device=V.device, dtype=V.dtype)
    T = V.size(1)
    out = torch.empty_like(V)
    c = W[2]
    out[:, 2:T - 2] = (c[0] * V[:, 0:T - 4] + c[1] * V[:, 1:T - 3] + c[2] * V[:, 2:T - 2] + c[3] * V[:, 3:T - 1]
                       + c[4] * V[:, 4:T])
    out[:, :2] = V[:, :5] @ W[:2].t()
    out[:, T - 2:] = V[:, T - 5:] @ W[3:].t()
    return out


def _get(cfg, path, default=None):
    """Read ``a.b.c`` from a nested dict / attribute config (DictConfig-like)."""
    cur = cfg
    for key in path.split("."):
        if cur is None:
            return default
        if isinstance(cur, dict):
            cur = cur.get(key, None)
        else:
            cur = getattr(cur, key, None)
    return default if cur is None else cur


def equation_terms(coefs, names, quantize=False, round_to=3) -> str:
    """Term string of ``convert_sindy_model_to_sympyjax_model_core`` (pkpd/utils.py:378-397):
    ``+{c}*term`` for every |c| > 1e-3, with numpy's shortest round-trip float formatting."""
    s = ""
    for j, c in enumerate(np.asarray(coefs, dtype=np.float64)):
        if np.abs(c) > RHS_COEF_EPS:
            if quantize:
                c = np.round(c, round_to)
            s += f"+{c}*" + names[j].replace(" ", "*")
    return s


def equation_string(joint_coefs, names, quantize=False, round_to=3) -> str:
    """``global_equation_string`` (sindy.py:276): 'Treatment 0: x_dot = ... | Treatment 1: ...'."""
    return " | ".join(f"Treatment {a}: x_dot = {equation_terms(c, names, quantize, round_to)}"
                      for a, c in enumerate(np.asarray(joint_coefs)))


def rhs_coefficients(joint_coefs, quantize=False, round_to=3) -> np.ndarray:
    """Coefficient table the sympy RHS evaluates: terms with |c| <= 1e-3 dropped, optionally
    rounded (the rounded value is what ``sympify`` of the string parses back)."""
    c = np.asarray(joint_coefs, dtype=np.float64).copy()
    keep = np.abs(c) > RHS_COEF_EPS
    if quantize:
        c = np.round(c, round_to)
    return np.where(keep, c, 0.0)


class SINDY:
    """MI355X drop-in for ``src.models.sindy.SINDY`` (EQ_4 PK/PD datasets, non-joint model)."""

    model_type = "sindy_regressor"
    tuning_criterion = "rmse"

    def __init__(self, args, dataset_collection=None, autoregressive=None, has_vitals=None, device=None, **kwargs):
        self.hparams = args
        self.dataset_collection = dataset_collection
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device()
                                                                                    if torch.cuda.is_available() else 0)
        m = lambda k, d=None: _get(args, f"model.{k}", d)   # noqa: E731
        self.lag_features = m("lag_features", 1)
        self.dim_outcome = int(m("dim_outcomes", 1))
        self.dim_treatments = int(m("dim_treatments", 2))
        self.dim_static_features = int(m("dim_static_features", 2))
        self.dim_vitals = int(m("dim_vitals", 0))
        self.smoother_kws = {"window_length": 5, "polyorder": 3}
        self.dt = float(m("dt", STANDARD_DT))   # reference hard-codes STANDARD_DT
        self.insite_val_error_threshold = m("insite_val_error_threshold")
        self.global_equation_string = ""
        self.sindy_threshold = float(m("sindy_threshold"))
        self.sindy_alpha = float(m("sindy_alpha"))
        self.smooth_input_data = bool(m("smooth_input_data", False))
        self.sindy_quantize = bool(m("sindy_quantize", False))
        self.sindy_quantize_global_model_round_to = int(m("sindy_quantize_global_model_round_to", 2))
        self.lam = m("lam")
        self.joint_model = bool(m("joint_model", False))
        self.insite = bool(m("insite", False))
        self.wsindy = bool(m("wsindy", False))
        self.use_smoothed_finite_difference = bool(m("use_smoothed_finite_difference", False))
        self.dataset_name = str(m("dataset_name", ""))
        # cancer_sim / EQ_5: treatment-segment split, FiniteDifference(order=1), one fit per arm of
        # the 4-valued treatment (sindy.py:160-183, 193-216, 289-312)
        self.segment_mode = "EQ_5" in self.dataset_name.upper() or "CANCER_SIM" in self.dataset_name.upper()
        self.ablation_more_complex_basis_functions = bool(m("ablation_more_complex_basis_functions", False))
        self.insight_recover_parametric_dist = bool(m("insight_recover_parametric_dist", False))
        self.treatment_mode = _get(args, "dataset.treatment_mode", "multiclass")
        self.projection_horizon = int(_get(args, "dataset.projection_horizon", 5))
        self.unscale_rmse = bool(_get(args, "exp.unscale_rmse", True))
        self.percentage_rmse = bool(_get(args, "exp.percentage_rmse", True))
        self.integrator = str(m("integrator", "euler5"))   # reference: Euler-5 (pkpd/utils.py:68-94)
        # BFGS status 3 -> global model (the code at sindy.py:628-631) or keep the iterate (the published
        # runs): default follows the published outputs
        self.insite_revert_on_zoom_fail = bool(m("insite_revert_on_zoom_fail", False))
        # PolynomialLibrary(**PolynomialLibrary_kw) of sindy.py:185-188
        self.lib_degree, self.lib_interaction_only = (4, False) if self.ablation_more_complex_basis_functions else (2, True)
        self.library = polynomial_library(self.dim_static_features, self.lib_degree, self.lib_interaction_only)
        self.feature_library_names = self.library.get_feature_names()
        self._roll_library = self.library   # the library the rollout evaluates (joint: folded per combination)
        self.feature_names = ["x0"] + [f"u{i}" for i in range(self.dim_static_features)]
        self.joint_coefs = None
        self.n_iter = None
        self._coef_dev = None
        self._check_supported()

    # ------------------------------------------------------------------ configuration checks
    def _check_supported(self):
        if not (self.segment_mode or "EQ_4" in self.dataset_name.upper()):
            raise NotImplementedError(f"dataset {self.dataset_name!r}: this build covers the PK/PD EQ_4 family and "
                                      "the treatment-segment datasets (cancer_sim, EQ_5_*)")
        if self.wsindy:
            raise NotImplementedError("weak SINDy (wsindy: true) is not on the MI355X path")
        if self.integrator not in ops.METHODS:
            raise ValueError(f"integrator must be one of {sorted(ops.METHODS)}")

    def prepare_data(self) -> None:
        c = self.dataset_collection
        if c is not None and not getattr(c, "processed_data_multi", True):
            c.process_data_multi()

    # ------------------------------------------------------------------ A1: DE format on device
    def _unscaled_inputs(self, dataset):
        sp = dataset.scaling_params
        d = dataset.data
        dev = self.device
        std, mean = float(sp["output_stds"]), float(sp["output_means"])
        prev = torch.as_tensor(np.ascontiguousarray(d["prev_outputs"][..., 0]), device=dev) * std + mean
        lo, hi = self.dim_outcome, self.dim_outcome + self.dim_static_features
        stat = (torch.as_tensor(np.ascontiguousarray(d["static_features"]), device=dev)
                * torch.as_tensor(np.asarray(sp["inputs_stds"][lo:hi], dtype=np.float64), device=dev)
                + torch.as_tensor(np.asarray(sp["input_means"][lo:hi], dtype=np.float64), device=dev))
        return prev, stat.contiguous(), std, mean

    def de_format(self, dataset, sequence_lengths_offset=1):
        """Device arrays of ``process_dataset_into_de_format`` (pkpd/utils.py:523-606): the
        reconstructed volume series x[N,T] (prev_outputs[:,0] ++ unscaled_outputs), statics u[N,U],
        the arm of each patient (current_treatments[:,0] == [1,0] -> 0, else 1; utils.py:425) and
        the discovery rows seq_len - offset (utils.py:426).  ``smooth_input_data`` smooths a copy
        the reference never reads back (utils.py:568-571), so it has no effect there or here."""
        d = dataset.data
        prev, stat, _, _ = self._unscaled_inputs(dataset)
        uo = torch.as_tensor(np.ascontiguousarray(d["unscaled_outputs"][..., 0]), device=self.device)
        x = torch.cat([prev[:, :1], uo], dim=1).contiguous()
        ct = torch.as_tensor(np.ascontiguousarray(d["current_treatments"][:, 0, :]), device=self.device)
        arm = torch.where((ct[:, 0] == 1) & (ct[:, 1] == 0), 0, 1).to(torch.int8)
        rows = (torch.as_tensor(np.asarray(d["sequence_lengths"]), device=self.device).to(torch.int64)
                - sequence_lengths_offset).to(torch.int32)
        return x, stat, arm, rows

    def de_format_segments(self, dataset):
        """Device arrays of the cancer_sim / EQ_5 branch of ``process_dataset_into_de_format``
        (pkpd/utils.py:607-637, sequence_lengths_offset = 0): the reconstructed series x[N, T], statics
        u[N, U], the per-step arm argmax(current_treatments) [N, T-1] (utils.py:624) and seq_len[N].
        The treatment-constant segments themselves are cut inside the Gram kernel."""
        d = dataset.data
        prev, stat, _, _ = self._unscaled_inputs(dataset)
        uo = torch.as_tensor(np.ascontiguousarray(d["unscaled_outputs"][..., 0]), device=self.device)
        x = torch.cat([prev[:, :1], uo], dim=1).contiguous()
        arm = torch.as_tensor(np.argmax(d["current_treatments"], axis=-1).astype(np.int8), device=self.device)
        sl = torch.as_tensor(np.asarray(d["sequence_lengths"]).astype(np.int32), device=self.device)
        return x, stat, arm.contiguous(), sl

    def _fit_segments(self, train_f):
        """cancer_sim / EQ_5 discovery (sindy.py:160-216): segment split + FD order 1 (or the
        savgol(2, 1)-smoothed variant) + library + per-arm Gram in one kernel, STLSQ per arm fused into
        the reduction launch (insite_sindy_fit_segments_f64)."""
        x, u, arm, sl = self.de_format_segments(train_f)
        fd = "smoothed1" if self.use_smoothed_finite_difference else "order1"
        if self.library.state_degree > 1:   # the degree-4 ablation library: per-arm power moments (insite_gen.hip)
            G, b = ops.gen_gram_segments(x, arm, sl, u, self.dt, self.library, n_arms=self.dim_treatments, fd=fd)
            coef, mask, iters = ops.stlsq(G, b, self.sindy_threshold, self.sindy_alpha, 100, True)
            return coef, mask, iters, G, b
        return ops.sindy_fit_segments(x, arm, sl, u, self.dt, self.library, self.sindy_threshold, self.sindy_alpha,
                                      max_iter=100, unbias=True, n_arms=self.dim_treatments, fd=fd)

    # ------------------------------------------------------------------ discovery
    def _fit_joint(self, train_f):
        """The joint ("one ODE") model (sindy.py:190, 203 with joint_model; DE format pkpd/utils.py:639-672):
        ONE regression over the rows x = unscaled_outputs[:seq_len - offset] (offset 1 for EQ_4, 0 for
        cancer_sim / EQ_5) with library inputs (x0, treatment bits, statics) — the multilabel treatments of
        ``dataset.treatment_mode=multilabel`` (run.py:198-201).  General one-state Gram + STLSQ on the GPU."""
        d = train_f.data
        ct = np.asarray(d["current_treatments"])
        if ct.ndim != 3 or ct.shape[-1] > 2 or not np.all((ct == 0) | (ct == 1)):
            raise NotImplementedError("joint_model needs binary multilabel treatments (dataset.treatment_mode="
                                      "multilabel, at most 2 treatment columns)")
        n_in = ct.shape[-1]
        self.library = polynomial_library(self.dim_static_features, self.lib_degree, self.lib_interaction_only,
                                          n_inputs=n_in)
        self.feature_library_names = self.library.get_feature_names()
        self.feature_names = list(self.library.input_names)
        _, stat, _, _ = self._unscaled_inputs(train_f)
        x = torch.as_tensor(np.ascontiguousarray(d["unscaled_outputs"][..., 0]), device=self.device)
        code = torch.as_tensor(self._treatment_code(ct), device=self.device)
        offset = 0 if self.segment_mode else 1
        rows = (torch.as_tensor(np.asarray(d["sequence_lengths"]), device=self.device).to(torch.int64) - offset)
        if self.segment_mode:
            fd, need = ("smoothed1" if self.use_smoothed_finite_difference else "order1"), 2
        else:
            fd, need = "smoothed4", 5
        if int(rows.min().item()) < need:
            raise ValueError(f"a training trajectory has fewer than {need} rows for the {fd} derivative")
        coef, mask, iters, _, _ = ops.gen_sindy_fit(x, stat, rows.to(torch.int32), self.dt, self.library,
                                                    self.sindy_threshold, self.sindy_alpha, step_in=code, fd=fd)
        return self._finish_fit(coef, mask, iters)

    @staticmethod
    def _treatment_code(ct) -> np.ndarray:
        """Per-step input code of binary multilabel treatments [N, T, n_in]: bit i = treatment i."""
        ct = np.asarray(ct)
        code = np.zeros(ct.shape[:2], dtype=np.int8)
        for i in range(ct.shape[-1]):
            code |= (ct[..., i].astype(np.int8) << i)
        return np.ascontiguousarray(code)

    def _fold_joint(self, rhs):
        """The joint RHS sum_j c_j x^e_j in(k)^tau_j m_j(u) as per-combination (arm) coefficients over the
        library with the input columns dropped: combination c keeps the columns whose inputs are all on in
        c (binary inputs), so the per-arm rollout kernels evaluate the same f(y, in_k, u)."""
        lib = self.library
        n_in, U = lib.n_inputs, lib.n_statics
        e = lib.exps
        keep_cols = [0] + list(range(1 + n_in, 1 + n_in + U))
        red_rows, index = [], []
        for row in e[:, keep_cols].tolist():
            if row not in red_rows:
                red_rows.append(row)
            index.append(red_rows.index(row))
        from .library import PolyLibrary
        red = PolyLibrary(np.array(red_rows, dtype=np.int8), (lib.input_names[0],) + tuple(lib.input_names[1 + n_in:]))
        NC = 1 << n_in
        folded = np.zeros((NC, len(red_rows)))
        tin = [(sum(1 << i for i in range(n_in) if e[j, 1 + i] > 0)) for j in range(lib.n_terms)]
        for c in range(NC):
            for j in range(lib.n_terms):
                if (tin[j] & ~c) == 0:
                    folded[c, index[j]] += rhs[0, j]
        return red, folded

    def fit(self, train_f, val_f=None):
        """Global discovery per arm (sindy.py:145-336): one Gram pass + STLSQ on the GPU."""
        self.prepare_data()
        if self.joint_model:
            return self._fit_joint(train_f)
        if self.segment_mode:
            coef, mask, iters, G, _ = self._fit_segments(train_f)
            empty = np.nonzero(G[:, 0, 0].cpu().numpy() == 0)[0]
            if empty.size:
                raise ValueError(f"treatment arm(s) {empty.tolist()} have no training segments "
                                 "(pysindy cannot fit an empty trajectory list)")
            return self._finish_fit(coef, mask, iters)
        x, u, arm, rows = self.de_format(train_f)
        if int(rows.min().item()) < 5:
            raise ValueError("a training trajectory has fewer than 5 rows: the savgol(5, 3) smoother "
                             "and the 5-point derivative need at least 5 samples")
        if self.library.state_degree > 1:     # the degree-4 ablation library: the general path
            coef, mask, iters, _, _ = ops.gen_sindy_fit(x, u, rows, self.dt, self.library, self.sindy_threshold,
                                                        self.sindy_alpha, group=arm, n_groups=self.dim_treatments,
                                                        fd="smoothed4")
            return self._finish_fit(coef, mask, iters)
        coef, mask, iters, _, _ = ops.sindy_fit(x, u, arm, rows, self.dt, self.library, self.sindy_threshold,
                                                self.sindy_alpha, max_iter=100, unbias=True,
                                                n_arms=self.dim_treatments, fd="smoothed4")
        return self._finish_fit(coef, mask, iters)

    def _finish_fit(self, coef, mask, iters):
        iters_h = iters.cpu().numpy()
        if np.any(iters_h < 0):
            raise np.linalg.LinAlgError("STLSQ ridge system is not positive definite")
        self.joint_coefs = coef.cpu().numpy()
        self.coef_mask = mask.cpu().numpy().astype(bool)
        self.n_iter = iters_h
        rhs = rhs_coefficients(self.joint_coefs, self.sindy_quantize, self.sindy_quantize_global_model_round_to)
        if self.joint_model:
            self._roll_library, rhs = self._fold_joint(rhs)
            self.global_equation_string = "Joint Model: x_dot = " + equation_terms(
                self.joint_coefs[0], self.feature_library_names, self.sindy_quantize,
                self.sindy_quantize_global_model_round_to)                           # sindy.py:285, 315
        else:
            self._roll_library = self.library
            self.global_equation_string = equation_string(self.joint_coefs, self.feature_library_names,
                                                          self.sindy_quantize, self.sindy_quantize_global_model_round_to)
        self._coef_dev = torch.as_tensor(np.ascontiguousarray(rhs), device=self.device)
        logger.info("[Model]: %s", self.global_equation_string)
        return self

    # ------------------------------------------------------------------ rollout (A8)
    def _predict_device(self, dataset, tau=1):
        """Standardised open-loop predictions [N, T-1] on the device (sindy.py:371-431); with
        ``insite`` the per-patient refined predictions (get_predictions passes the reference's default
        projection_horizon=1, the autoregressive path the dataset's tau; sindy.py:362-369, 736-738)."""
        if self.insite:
            return self._refined_device(dataset, tau)
        if self._coef_dev is None:
            raise RuntimeError("fit() first")
        d = dataset.data
        prev, stat, std, mean = self._unscaled_inputs(dataset)
        T = d["prev_outputs"].shape[1]
        if self.joint_model:   # per-step treatment combination = the folded model's arm
            arm = torch.as_tensor(self._treatment_code(d["current_treatments"]), device=self.device)
        else:
            arm = torch.as_tensor(np.argmax(d["current_treatments"], axis=-1).astype(np.int8), device=self.device)
        y = ops.rollout(prev[:, 0].contiguous(), stat, arm.contiguous(), self._coef_dev, self._roll_library, self.dt,
                        method=self.integrator, drop_below=0.0, T=T)
        return (y - mean) / std

    def _refined_device(self, dataset, tau):
        """INSITE predictions (sindy.py:433-715): every row with sequence_length > tau refines the active
        global coefficients by BFGS on its own observed prefix (insite_refine_f64, one lane per row),
        then rolls its refined model out with the reference's Euler-5 odeint.  Standardised [N, T]."""
        if self.joint_coefs is None:
            raise RuntimeError("fit() first")
        if self.lam is None:
            raise ValueError("model.lam must be set for insite: true (reference config: 10.0 for EQ_4)")
        d = dataset.data
        prev, stat, std, mean = self._unscaled_inputs(dataset)
        if self.smooth_input_data:      # applied here in the reference (sindy.py:557-560), unlike the DE format
            prev = savgol_5_3_rows(prev)
        if self.segment_mode and "EQ_5" in self.dataset_name.upper() and stat.shape[1] >= 2:
            # the reference's EQ_5 refinement binds u1 to static_features[0] (sindy.py:536), unlike its
            # global-model rollout (sindy.py:302): kept, so refined EQ_5 predictions match the reference
            stat = stat[:, :1].expand(-1, stat.shape[1]).contiguous()
        if self.joint_model:   # the per-step treatment bit code selects the folded combination (sindy.py:469-551)
            arm = torch.as_tensor(self._treatment_code(d["current_treatments"]), device=self.device)
        else:
            arm = torch.as_tensor(np.argmax(d["current_treatments"], axis=-1).astype(np.int8), device=self.device)
        sl = torch.as_tensor(np.asarray(d["sequence_lengths"]).astype(np.int32), device=self.device)
        preds, coef, status, iters = ops.insite_refine(prev.contiguous(), arm.contiguous(), stat, sl, self.joint_coefs,
                                                       self.library, self.dt, float(self.lam), int(tau), substeps=5,
                                                       revert_on_zoom_fail=self.insite_revert_on_zoom_fail)
        self.insite_status, self.insite_iters, self.insite_coefs = status, iters, coef
        scaled = ((preds - mean) / std).contiguous()
        # the reference refuses refined predictions with NaN or Inf (sindy.py:710): a refined model that blows up
        # inside the row's horizon ends the run there, not in a metric later
        if not bool(torch.isfinite(scaled).all()):
            raise AssertionError("Scaled_preds contains NaN or Inf")
        return scaled

    def get_predictions(self, dataset) -> np.ndarray:
        logger.info("Predictions for %s.", getattr(dataset, "subset_name", "?"))
        p = self._predict_device(dataset).cpu().numpy()[..., None]
        assert not np.any(np.isnan(p)), "Predictions contains NaN"
        return p

    def _slice_device(self, pred, dataset, offset=1):
        """tau-step window per row from max(offset, seq_len - tau) (sindy.py:729-733), with
        jax.lax.dynamic_slice's clamp to [0, T - tau]."""
        tau = self.projection_horizon
        T = pred.shape[1]
        sl = torch.as_tensor(np.asarray(dataset.data["sequence_lengths"]).astype(np.int64), device=pred.device)
        lo = torch.clamp(torch.clamp(sl - tau, min=offset), 0, T - tau)
        idx = lo[:, None] + torch.arange(tau, device=pred.device)[None, :]
        return torch.gather(pred, 1, idx)

    def get_autoregressive_predictions(self, dataset) -> np.ndarray:
        logger.info("Autoregressive Prediction for %s.", getattr(dataset, "subset_name", "?"))
        pred = self._predict_device(dataset, tau=self.projection_horizon)
        return self._slice_device(pred, dataset).cpu().numpy()[..., None]

    # ------------------------------------------------------------------ metrics (A10)
    def _sse(self, pred_scaled, target, active, std, mean):
        """Masked squared-error sums on the device; the prediction is un-scaled in the kernel
        (pred * std + mean, as time_varying_model.py:249) when ``unscale_rmse``."""
        tgt = torch.as_tensor(np.ascontiguousarray(target), device=pred_scaled.device)
        act = torch.as_tensor(np.ascontiguousarray(active), device=pred_scaled.device)
        if self.unscale_rmse:
            return ops.masked_sse(pred_scaled.contiguous(), tgt, act, scale=std, shift=mean)
        return ops.masked_sse(pred_scaled.contiguous(), tgt, act)

    def get_normalised_masked_rmse(self, dataset, one_step_counterfactual=False):
        logger.info("RMSE calculation for %s.", getattr(dataset, "subset_name", "?"))
        sp = dataset.scaling_params
        std, mean = float(sp["output_stds"]), float(sp["output_means"])
        pred = self._predict_device(dataset)
        if torch.isnan(pred).any():
            raise AssertionError("Predictions contains NaN")
        key = "unscaled_outputs" if self.unscale_rmse else "outputs"
        per, cnt, last = self._sse(pred, dataset.data[key][..., 0], dataset.data["active_entries"][..., 0], std, mean)
        per, cnt, last = per.cpu().numpy(), cnt.cpu().numpy(), last.cpu().numpy()
        norm = dataset.norm_const
        scale = 100.0 if self.percentage_rmse else 1.0
        with np.errstate(invalid="ignore", divide="ignore"):
            orig = np.sqrt((per / cnt).mean()) / norm * scale
            allv = np.sqrt(per.sum() / cnt.sum()) / norm * scale
            if not one_step_counterfactual:
                return orig, allv
            lastv = np.sqrt(last[0] / last[1]) / norm * scale
        return orig, allv, lastv

    def get_normalised_n_step_rmses(self, dataset, datasets_mc=None):
        logger.info("RMSE calculation for %s.", getattr(dataset, "subset_name", "?"))
        seq = dataset.data_processed_seq
        assert seq is not None, "dataset has no data_processed_seq (process_data_multi first)"
        sp = dataset.scaling_params
        std, mean = float(sp["output_stds"]), float(sp["output_means"])
        pred = self._slice_device(self._predict_device(dataset if datasets_mc is None else datasets_mc,
                                                       tau=self.projection_horizon), dataset)
        key = "unscaled_outputs" if self.unscale_rmse else "outputs"
        not_nan = ~np.isnan(seq["outputs"][..., 0]).any(axis=1)          # time_varying_model.py:302-303
        idx = torch.as_tensor(np.nonzero(not_nan)[0], device=pred.device)
        per, cnt, _ = self._sse(pred.index_select(0, idx), seq[key][not_nan][..., 0],
                                seq["active_entries"][not_nan][..., 0], std, mean)
        per, cnt = per.cpu().numpy(), cnt.cpu().numpy()
        r = np.sqrt(per / cnt) / dataset.norm_const
        return r * (100.0 if self.percentage_rmse else 1.0)
