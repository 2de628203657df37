#!/usr/bin/env python3
"""Extract the reference's published per-run results for the PK/PD path into a JSON fixture.

Sources (data, read as text): the ``[Exp evaluation complete] {...}`` log lines the reference's
``run.py:121`` writes in ``/root/reference/results/2_main_table/final_with_insite.txt`` (every dataset --
EQ_4_*, cancer_sim, EQ_5_* -- and method in {sindy, insite}: the first seed-1 line, seed 1 being the
logged ``exp.seed`` of the cohort) and in the one-ODE ablation log
``results/ablation/one_ode/build_tables/run_ct-20230516-043331_insite-sindy_cancer_sim_1_5-runs_log_one_big_ode.txt``
(joint model, multilabel treatments: every seed, keys ``ABLATION_ONE_ODE/<dataset>/<method>/<seed>``),
each with its line number.  Output:
``tests/golden/reference_log_anchors.json`` (committed; the GPU box never reads the reference).

    python tests/golden/extract_log_anchors.py
"""
from __future__ import annotations

import ast
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/results/2_main_table/final_with_insite.txt"
SRC_ONE_ODE = ("/root/reference/results/ablation/one_ode/build_tables/"
               "run_ct-20230516-043331_insite-sindy_cancer_sim_1_5-runs_log_one_big_ode.txt")
KEYS = ("encoder_test_rmse_all", "encoder_test_rmse_orig", "encoder_test_rmse_last", "decoder_test_rmse_2-step",
        "decoder_test_rmse_3-step", "decoder_test_rmse_4-step", "decoder_test_rmse_5-step",
        "decoder_test_rmse_6-step", "global_equation_string", "seconds_taken", "method", "seed")


def main():
    marker = "[Exp evaluation complete] "
    out = {}
    with open(SRC) as f:
        for no, line in enumerate(f, 1):
            if marker not in line:
                continue
            rec = ast.literal_eval(line.split(marker, 1)[1].strip())
            ds, m = rec.get("dataset_name", ""), rec.get("method")
            if m not in ("sindy", "insite") or rec.get("seed") != 1:
                continue
            key = f"{ds}/{m}"
            if key not in out:
                out[key] = {"source": f"results/2_main_table/final_with_insite.txt:{no}",
                            **{k: rec[k] for k in KEYS if k in rec}}
    with open(SRC_ONE_ODE) as f:
        for no, line in enumerate(f, 1):
            if marker not in line:
                continue
            rec = ast.literal_eval(line.split(marker, 1)[1].strip())
            key = f"ABLATION_ONE_ODE/{rec['dataset_name']}/{rec['method']}/{rec['seed']}"
            out[key] = {"source": f"results/ablation/one_ode/build_tables/{os.path.basename(SRC_ONE_ODE)}:{no}",
                        **{k: rec[k] for k in KEYS if k in rec}}
    path = os.path.join(HERE, "reference_log_anchors.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"wrote {path}: {sorted(out)}")


if __name__ == "__main__":
    main()
