"""Stopping-control sweep of the INSITE refinement restatement against the published runs.

Test / diagnostic infrastructure only (runs the CPU oracle).  The reference calls
``jax.scipy.optimize.minimize(f_to_min, c0, method='BFGS', tol=1e-12)`` (sindy.py:627) and reverts status 3 to c0
(sindy.py:628-631); jax's ``minimize`` does not forward ``tol``, so ``minimize_bfgs`` runs with gtol = 1e-5 on the
gradient's inf-norm, maxiter = 200 * size and line_search maxiter = 10 (oracle/insite_refine_ref.py header).  This
sweeps those controls, and which statuses revert, on the regenerated EQ_5_B / EQ_5_D cohorts, the one-ODE joint cohort
and (the constraint) EQ_4_B, and reports for every setting the relative difference of every published one-step metric
(final_with_insite.txt:2362-2392; the one-ODE log) plus the window / last-entry SSE split of the one-step set.

    python tools/insite_stop_sweep.py [--out profiles/r05/insite_stop_sweep.json] [--only NAME ...]
"""
import argparse
import json
import os
import sys
import time
import warnings
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import cancer_sim_ref as CS            # noqa: E402
from oracle import insite_ref as R                 # noqa: E402
from oracle import insite_refine_ref as Q          # noqa: E402
from oracle import ref_cohort as RC                # noqa: E402

ANCH = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_log_anchors.json")))

SETTINGS = [("base", {})]
SETTINGS += [(f"gtol={g:g}", {"gtol": g}) for g in (1e-2, 3e-3, 1e-3, 3e-4, 1e-4, 3e-5, 1e-6, 1e-7)]
SETTINGS += [(f"maxiter={m}", {"maxiter": m}) for m in (1, 2, 3, 4, 6, 10)]
SETTINGS += [(f"ls_maxiter={m}", {"ls_maxiter": m}) for m in (1, 2, 3, 5)]
SETTINGS += [("revert={3}", {"revert_statuses": {3}}), ("revert={5}", {"revert_statuses": {5}}),
             ("revert={1,2,3,4,5}", {"revert_statuses": {1, 2, 3, 4, 5}})]


def _rows(args):
    prev, arms, stat, sl, c0, exps, tau, n_inputs, dt, kw = args
    out, st = [], []
    for i in range(prev.shape[0]):
        p, _, s, _ = Q.refine_patient(prev[i], arms[i], stat[i], int(sl[i]), c0, exps, dt, 10.0, tau,
                                      n_inputs=n_inputs, **kw)
        out.append(p)
        st.append(s)
    return np.stack(out), np.array(st)


def _split(P, one, nc, log_all, log_last):
    act = one.data["active_entries"][..., 0]
    tgt = one.data["unscaled_outputs"][..., 0]
    last = act - np.concatenate([act[:, 1:], np.zeros((act.shape[0], 1))], axis=1)
    ins = act - last
    a_ = (log_all * nc / 100) ** 2 * act.sum()
    l_ = (log_last * nc / 100) ** 2 * last.sum()
    w = float((((P - tgt) ** 2) * ins).sum())
    lst = float((((P - tgt) ** 2) * last).sum())
    return {"window_sse_rel": w / (a_ - l_) - 1.0, "last_sse_rel": lst / l_ - 1.0}


def cases():
    """(name, one-step subset, c0, exps, statics, arms, n_inputs, dt, normaliser, log anchors)."""
    out = []
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        for eq in ("EQ_5_B", "EQ_5_D"):
            coll = CS.make_collection(1, equation=eq)
            pipe = CS.sindy_pipeline(coll)
            one = coll["test_cf_one_step"]
            U = one.data["static_features"].shape[-1]
            prev, st = R.unscale_inputs(one.data, one.scaling_params, 1, U)
            if U >= 2:
                st = np.repeat(st[:, :1], U, axis=1)       # sindy.py:536
            out.append((eq, one, prev, pipe["joint_coefs"], pipe["exps"], st,
                        np.argmax(one.data["current_treatments"], axis=-1), 0, R.STANDARD_DT,
                        CS.TUMOUR_DEATH_THRESHOLD, ANCH[f"{eq}/insite"]))
        coll = CS.make_collection(10, treatment_mode="multilabel")
        pipe = CS.joint_pipeline(coll)
        one = coll["test_cf_one_step"]
        prev, st = R.unscale_inputs(one.data, one.scaling_params, 1, 1)
        tr = np.asarray(one.data["current_treatments"])
        out.append(("one_ode_joint", one, prev, pipe["joint_coefs"], pipe["exps"], st,
                    (tr[..., 0] + 2 * tr[..., 1]).astype(np.int64), 2, R.STANDARD_DT, CS.TUMOUR_DEATH_THRESHOLD,
                    ANCH["ABLATION_ONE_ODE/cancer_sim/insite/1"]))
    coll = RC.make_collection("EQ_4_B")
    c0 = R.sindy_pipeline({"train": coll["train"]}, dt=R.STANDARD_DT)["joint_coefs"]
    one = coll["test_cf_one_step"]
    prev, st = R.unscale_inputs(one.data, one.scaling_params)
    out.append(("EQ_4_B", one, prev, c0, R.poly_library(3, 2, True), st,
                np.argmax(one.data["current_treatments"], axis=-1), 0, R.STANDARD_DT, None, ANCH["EQ_4_B/insite"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05", "insite_stop_sweep.json"))
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--workers", type=int, default=min(8, os.cpu_count() or 1))
    a = ap.parse_args()
    cs = cases()
    res = {}
    keys = ["encoder_test_rmse_orig", "encoder_test_rmse_all", "encoder_test_rmse_last"]
    with ProcessPoolExecutor(a.workers) as ex:
        for name, kw in SETTINGS:
            if a.only and name not in a.only:
                continue
            res[name] = {}
            for (cn, one, prev, c0, exps, st, arms, n_in, dt, nc, log) in cs:
                t0 = time.time()
                sl = one.data["sequence_lengths"].astype(np.int64)
                chunks = np.array_split(np.arange(prev.shape[0]), 64)
                parts = list(ex.map(_rows, [(prev[c], arms[c], st[c], sl[c], c0, exps, 1, n_in, dt, kw)
                                            for c in chunks]))
                P = np.concatenate([p for p, _ in parts])
                S = np.concatenate([s for _, s in parts])
                kwm = {} if nc is None else {"norm_const": nc}
                m = R.masked_rmse(P[..., None], one.data["unscaled_outputs"], one.data["active_entries"],
                                  one_step_counterfactual=True, **kwm)
                rel = {k: float(v / log[k] - 1.0) for k, v in zip(keys, m)}
                d = {"rel": rel, "statuses": {int(s): int((S == s).sum()) for s in np.unique(S)}}
                d.update(_split(P, one, nc if nc is not None else R.MAX_VALUE, log[keys[1]], log[keys[2]]))
                res[name][cn] = d
                print(f"{name:22s} {cn:14s} " + " ".join(f"{k[18:]}={v:+.2e}" for k, v in rel.items())
                      + f" win={d['window_sse_rel']:+.3f} last={d['last_sse_rel']:+.3f} st={d['statuses']}"
                      + f" ({time.time() - t0:.0f}s)", flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
