#!/bin/bash
# Iteration loop: gpu tests, step timings (default + ablation builds), graph-mode bench under a kernel trace.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${PYTEST_EXTRA:-} > gpurun_out/t_all.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/t_all.log | head -40; tail -5 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
TV_RUNS="step:--layout time_bits${KB_EXTRA:-}" ITERS=50 bash tools/g_tv.sh
MODE=graph bash tools/g_trace.sh
python tools/trace_gaps.py gpurun_out/tr_graph/run_kernel_trace.csv 30 9
