"""Config composition for the SINDy/INSITE plugin (Hydra-style, no Hydra dependency).

Mirrors what the reference builds per run (``run.py:196-268`` + ``compose(config_name='ct_config',
overrides=...)``): the experiment defaults, ``+backbone=<name>`` and ``+dataset=<name>`` groups from
``insite_amd/configs/``, then dotted ``a.b.c=value`` overrides (values parsed as YAML scalars).
The result is a plain nested dict; ``SINDY`` reads it with dotted paths like the reference reads
its DictConfig.
"""
from __future__ import annotations

import copy
import os

import yaml

CONFIG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "configs")


def _load(rel: str) -> dict:
    path = os.path.join(CONFIG_DIR, rel)
    if not os.path.exists(path):
        raise FileNotFoundError(f"no config {rel!r} under {CONFIG_DIR}")
    with open(path) as f:
        return yaml.safe_load(f) or {}


def merge(base: dict, extra: dict) -> dict:
    """Recursive merge: values of ``extra`` win; nested dicts merge key by key."""
    out = copy.deepcopy(base)
    for k, v in extra.items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def set_path(cfg: dict, dotted: str, value) -> None:
    cur = cfg
    keys = dotted.split(".")
    for k in keys[:-1]:
        if not isinstance(cur.get(k), dict):
            cur[k] = {}
        cur = cur[k]
    cur[keys[-1]] = value


def get_path(cfg: dict, dotted: str, default=None):
    cur = cfg
    for k in dotted.split("."):
        if not isinstance(cur, dict) or k not in cur:
            return default
        cur = cur[k]
    return cur


def compose(overrides=()) -> dict:
    """Experiment defaults + ``+group=name`` config groups + ``key=value`` overrides."""
    cfg = _load("experiment.yaml")
    plain = []
    for o in overrides:
        if o.startswith("+") and "=" in o:
            group, name = o[1:].split("=", 1)
            cfg = merge(cfg, _load(os.path.join(group, f"{name}.yaml")))
        else:
            plain.append(o)
    for o in plain:
        if "=" not in o:
            raise ValueError(f"override {o!r} is not key=value")
        k, v = o.split("=", 1)
        set_path(cfg, k, yaml.safe_load(v) if v != "" else None)
    if get_path(cfg, "dataset.seed") is None and get_path(cfg, "dataset") is not None:
        set_path(cfg, "dataset.seed", get_path(cfg, "exp.seed", 0))
    return cfg


def driver_config() -> dict:
    """The experiment-driver settings (``configs/config.yaml``)."""
    return _load("config.yaml")


def run_overrides(driver: dict, dataset_name: str, method_name: str, seed: int, domain_conf) -> list:
    """The override list the reference's ``run_exp_ct`` builds for the SINDy family on EQ_4
    datasets (run.py:184-268): thresholds / lam picked by dataset-name substring."""
    dp = driver["sindy"]["dataset_params"]
    thr = [v for k, v in dp["sindy_threshold"].items() if k in dataset_name]
    lam = [v for k, v in dp["lam"].items() if k in dataset_name]
    if len(thr) != 1 or len(lam) != 1:
        raise ValueError("Must only specify one sindy threshold / lam for " + dataset_name)
    run = driver["run"]
    if "EQ_4" not in dataset_name:
        raise NotImplementedError(f"dataset {dataset_name!r}: only the PK/PD EQ_4 family is on the MI355X path")
    return [f"+backbone={method_name}", f"exp.seed={seed}",
            f"dataset.num_patients.train={run['train_samples']}", f"dataset.num_patients.val={run['val_samples']}",
            f"dataset.num_patients.test={run['test_samples']}", f"dataset.coeff={domain_conf}",
            "+dataset=pkpd_sim", f"dataset.equation_str={dataset_name}", f"model.dataset_name={dataset_name}",
            f"model.sindy_threshold={thr[0]}", f"model.sindy_alpha={driver['sindy']['sindy_alpha']}",
            f"model.lam={lam[0]}", "dataset.treatment_mode=multiclass"]
