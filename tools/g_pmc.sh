#!/bin/bash
# HBM traffic counters (separate --pmc passes, one counter group each; MI355X_MICROARCH.md HBM section):
# the C2 rollout and gram kernels via tools/kbench.py, plus the access-pattern probe as a known-byte
# calibration of 8-B-per-lane streaming reads/writes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for C in FETCH_SIZE WRITE_SIZE; do
  for OP in "rollout --layout time_bits" "gram --layout time" "sindy_fit --layout time"; do
    tag=$(echo "$OP" | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $C -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/${tag}_$C" -o run --output-format csv -- python3 tools/kbench.py --op $OP --iters 10 > gpurun_out/pmc/${tag}_$C.log 2>&1 || exit 1
  done
  timeout -s KILL 60 rocprofv3 --pmc $C -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/probe_$C" -o run --output-format csv -- ./tools/probe/bin/layout_probe 100000 200 > gpurun_out/pmc/probe_$C.log 2>&1 || exit 1
done
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.json && echo ALLOK
