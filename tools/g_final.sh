#!/bin/bash
# Round-end evidence: full GPU suite, smoke, the default bench line (as the driver runs it) and its
# rocprofv3 kernel summary.  Every GPU step has its own time limit; the first failure ends the call.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.log 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/bench_prof.log 2>&1 || { tail -20 $O/bench_prof.log; exit 1; }
# the per-symbol stats mix the 100k x 200 step launches with the 1M x 500 north-star probe: split by grid
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
[ -n "$T" ] && python tools/rocprof_by_grid.py "$T" $O/bench_kernels_by_grid.csv && head -12 $O/bench_kernels_by_grid.csv
timeout -k 10 300 python bench.py --no-cpu-baseline --no-north-star --mode fused > $O/fused.log 2>$O/fused.err || { tail -20 $O/fused.err; exit 1; }
tail -1 $O/fused.log | cut -c1-300
echo ALLOK
