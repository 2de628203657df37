#!/bin/bash
# One GPU round: gpu tests, smoke, bench (JSON line), rocprofv3 kernel stats of the same bench.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${PYTEST_EXTRA:-} > gpurun_out/t_all.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/t_all.log | head -40; tail -5 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-north-star > gpurun_out/bench_prof.log 2>&1 || { tail -20 gpurun_out/bench_prof.log; exit 1; }
tail -1 gpurun_out/bench_prof.log
find gpurun_out/prof -name "*stats*"
