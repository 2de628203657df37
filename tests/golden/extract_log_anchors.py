#!/usr/bin/env python3
"""Extract the reference's published per-run results for the PK/PD path into a JSON fixture.

Source (data, read as text): ``/root/reference/results/2_main_table/final_with_insite.txt`` — the
``[Exp evaluation complete] {...}`` log lines the reference's ``run.py:121`` writes.  For every
EQ_4_* dataset and method in {sindy, insite} the first seed-1 line is kept (seed 1 is the logged
``exp.seed`` of the cohort) with its line number.  Output:
``tests/golden/reference_log_anchors.json`` (committed; the GPU box never reads the reference).

    python tests/golden/extract_log_anchors.py
"""
from __future__ import annotations

import ast
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/results/2_main_table/final_with_insite.txt"
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
            if not ds.startswith("EQ_4") or m not in ("sindy", "insite") or rec.get("seed") != 1:
                continue
            key = f"{ds}/{m}"
            if key not in out:
                out[key] = {"source": f"results/2_main_table/final_with_insite.txt:{no}",
                            **{k: rec[k] for k in KEYS if k in rec}}
    path = os.path.join(HERE, "reference_log_anchors.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"wrote {path}: {sorted(out)}")


if __name__ == "__main__":
    main()
