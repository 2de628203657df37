#!/bin/bash
# time_variants over several op/args sets, summarised
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
: > gpurun_out/tv.log
IFS='|' read -ra RUNS <<< "$TV_RUNS"
for r in "${RUNS[@]}"; do
  OP=${r%%:*} EXTRA_SETS="${r#*:}" ITERS=${ITERS:-30} bash tools/time_variants.sh >> gpurun_out/tv.log 2>&1 || exit 1
done
python - <<'PY'
import json
for l in open("gpurun_out/tv.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["op"], d["patients"], d["T"], d["layout"], d.get("cold"), d["lib"].split("/")[-1], round(d["ms_per_call"] * 1e3, 1))
PY
