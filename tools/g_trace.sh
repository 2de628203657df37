#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
M=${MODE:-graph}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/tr_$M" -o run --output-format csv -- python3 bench.py --mode $M --no-cpu-baseline --no-north-star --steps 50 ${BENCH_EXTRA:-} > gpurun_out/tr_$M.log 2>&1 || { tail -20 gpurun_out/tr_$M.log; exit 1; }
tail -1 gpurun_out/tr_$M.log
