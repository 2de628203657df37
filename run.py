#!/usr/bin/env python3
"""Experiment entry point: the reference's ``run.py`` + ``train_sindy.main`` for the SINDy
backbone on the PK/PD EQ_4 datasets, with discovery and rollouts on MI355X.

Mirrors ``run.py:100-294`` (run list over datasets x methods x seeds, ``[Exp evaluation complete]``
log line per run, ``{'errored': True}`` on failure outside debug mode) and
``libs_m/ct/runnables/train_sindy.py:21-113`` (collection -> ``process_data_multi`` -> model dims ->
``SINDY(args, collection).fit`` -> one-step counterfactual RMSEs -> tau-step RMSEs -> equation).

    python run.py                                   # configs/config.yaml run list
    python run.py --datasets EQ_4_C --seeds 0 1     # subset of the main table
    python run.py +backbone=sindy +dataset=pkpd_sim dataset.equation_str=EQ_4_A \\
                  model.dataset_name=EQ_4_A model.sindy_threshold=0.1 model.sindy_alpha=0.5 \\
                  dataset.num_patients.train=1000 dataset.num_patients.val=100 dataset.num_patients.test=100
"""
from __future__ import annotations

import argparse
import logging
import os
import sys
import time
import traceback

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from insite_amd import config as C  # noqa: E402

logger = logging.getLogger("insite_amd.run")


def train_sindy_main(args: dict, dataset_name: str = "", device=None) -> dict:
    """``train_sindy.main`` (train_sindy.py:21-113)."""
    from insite_amd import pkpd
    from insite_amd.sindy import SINDY
    results = {}
    seed = int(C.get_path(args, "exp.seed", 0))
    torch.manual_seed(seed)
    np.random.seed(seed)
    ds = args["dataset"]
    coll = pkpd.SyntheticPkpdDatasetCollection(conf_coeff=float(ds["coeff"]), num_patients=ds["num_patients"],
                                               equation_str=ds["equation_str"], seed=int(ds["seed"]),
                                               max_seq_length=int(ds.get("max_seq_length", 60)),
                                               projection_horizon=int(ds.get("projection_horizon", 5)),
                                               device=device, rng=str(ds.get("rng", "threefry")))
    coll.process_data_multi()
    tr = coll.train_f.data
    C.set_path(args, "model.dim_outcomes", tr["outputs"].shape[-1])
    C.set_path(args, "model.dim_treatments", tr["current_treatments"].shape[-1])
    C.set_path(args, "model.dim_vitals", 0)
    C.set_path(args, "model.dim_static_features", tr["static_features"].shape[-1])
    C.set_path(args, "model.treatment_mode", ds.get("treatment_mode", "multiclass"))
    model = SINDY(args, coll, device=device)
    model.fit(coll.train_f, coll.val_f)
    if model.insight_recover_parametric_dist:
        model.get_predictions(coll.val_f)
    o, a, last = model.get_normalised_masked_rmse(coll.test_cf_one_step, one_step_counterfactual=True)
    logger.info(f"Test normalised RMSE (all): {a}; Test normalised RMSE (orig): {o}; "
                f"Test normalised RMSE (only counterfactual): {last}")
    results.update({"encoder_test_rmse_all": a, "encoder_test_rmse_orig": o, "encoder_test_rmse_last": last})
    rm = model.get_normalised_n_step_rmses(coll.test_cf_treatment_seq)
    test_rmses = {f"{k + 2}-step": v for k, v in enumerate(rm)}
    logger.info(f"Test normalised RMSE (n-step prediction): {test_rmses}")
    results.update({"decoder_test_rmse_" + k: v for k, v in test_rmses.items()})
    results.update({"global_equation_string": model.global_equation_string, "fine_tuned": model.insite})
    return results


def run_one(driver: dict, dataset_name: str, method_name: str, seed: int, domain_conf, extra=(), device=None):
    """``run_exp_wrapper_outer`` (run.py:139-169)."""
    logger.info(f"[Now evaluating exp] {(dataset_name, method_name, seed, domain_conf)}")
    t0 = time.perf_counter()
    try:
        args = C.compose(C.run_overrides(driver, dataset_name, method_name, seed, int(domain_conf)) + list(extra))
        result = train_sindy_main(args, dataset_name=dataset_name, device=device)
        # run_exp_ct's tail (reference run.py:305-306): method, seed, seconds_taken (wall time of the run)
        result.update({"method": method_name, "seed": seed, "seconds_taken": time.perf_counter() - t0})
        result["errored"] = False
    except Exception as e:  # noqa: BLE001 - mirrors the reference's catch-all outside debug mode
        if driver["setup"].get("debug_mode", True):
            raise
        logger.exception(f"[Error] {e}")
        logger.info(f"[Failed evaluating exp] {(dataset_name, method_name, seed, domain_conf)}\t| error={e}")
        traceback.print_exc()
        result = {"errored": True}
    # run_exp_wrapper_outer's keys (reference run.py:170), in the logged order -- a failed run keeps its seed
    result.update({"dataset_name": dataset_name, "seed": seed, "method_name": method_name, "domain_conf": domain_conf})
    return result


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--datasets", nargs="*", default=None)
    ap.add_argument("--methods", nargs="*", default=None)
    ap.add_argument("--seeds", nargs="*", type=int, default=None)
    ap.add_argument("--domain-conf", type=float, default=None)
    ap.add_argument("--device", default=None)
    ap.add_argument("--no-debug", action="store_true", help="record failed runs as {'errored': True}")
    ap.add_argument("overrides", nargs="*", help="hydra-style overrides (+group=name, a.b=c)")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(levelname)s %(message)s")
    driver = C.driver_config()
    if a.no_debug:
        driver["setup"]["debug_mode"] = False
    results = []
    t0 = time.perf_counter()
    if any(o.startswith("+backbone=") for o in a.overrides):
        # single composed run, like `compose(config_name='ct_config', overrides=...)`
        args = C.compose(a.overrides)
        name = C.get_path(args, "dataset.equation_str")
        t1 = time.perf_counter()
        r = train_sindy_main(args, dataset_name=name, device=a.device)
        mname = C.get_path(args, "model.name", "").lower()
        r.update({"method": mname, "seed": C.get_path(args, "exp.seed", 0), "seconds_taken": time.perf_counter() - t1,
                  "errored": False, "dataset_name": name, "method_name": mname})
        results.append(r)
        logger.info(f"[Exp evaluation complete] {_printable(r)}")
    else:
        s = driver["setup"]
        datasets = a.datasets or s["datasets_to_evaluate"]
        methods = a.methods or s["methods_to_evaluate"]
        seeds = a.seeds if a.seeds is not None else list(range(s["seed_start"], s["seed_start"] + s["seed_runs"]))
        dc = a.domain_conf if a.domain_conf is not None else driver["run"]["domain_conf"]
        for dn in datasets:
            for seed in seeds:
                for mn in methods:
                    r = run_one(driver, dn, mn, seed, dc, a.overrides, device=a.device)
                    logger.info(f"[Exp evaluation complete] {_printable(r)}")
                    results.append(r)
    dt = time.perf_counter() - t0
    logger.info(f"Time taken for all runs: {dt}s\t| {dt / 60.0} minutes")
    return results


def _printable(r: dict) -> dict:
    return {k: (v.tolist() if isinstance(v, np.ndarray) else (float(v) if isinstance(v, np.floating) else v))
            for k, v in r.items()}


if __name__ == "__main__":
    main()
