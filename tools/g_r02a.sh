#!/bin/bash
# round-2 GPU pass: full -m gpu suite, smoke, headline bench, its rocprofv3 kernel stats, C5 bench.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r02a
O=gpurun_out/r02a
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.log 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-north-star --no-cpu-baseline > $O/bench_prof.log 2>&1 || { tail -20 $O/bench_prof.log; exit 1; }
timeout -k 10 300 python bench.py --config c5 > $O/c5.log 2>$O/c5.err || { tail -20 $O/c5.err; exit 1; }
echo ALLOK
