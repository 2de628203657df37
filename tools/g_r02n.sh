#!/bin/bash
# full GPU suite + C2 bench (two-stream pipeline, in-launch gram reduction) + kernel trace/stats
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02n}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2.log 2>$O/c2.err || { tail -20 $O/c2.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-north-star > $O/c2_prof.log 2>&1 || { tail -20 $O/c2_prof.log; exit 1; }
echo ALLOK
