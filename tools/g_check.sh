#!/bin/bash
# full GPU parity suite, then the F2 (insite) and default C2 bench lines
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 300 python bench.py --config insite > gpurun_out/ins.log 2>&1 || { tail -20 gpurun_out/ins.log; exit 1; }
tail -1 gpurun_out/ins.log | cut -c1-600
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-400
