#!/bin/bash
# round-2 GPU pass b: the general one-state path + the full suite, then C4 at T = 60 and 500.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_general.py -x -q --timeout 200 --timeout-method thread > $O/general.log 2>&1 || { tail -60 $O/general.log; exit 1; }
tail -2 $O/general.log
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --config c4 > $O/c4_T60.log 2>$O/c4_T60.err || { tail -20 $O/c4_T60.err; exit 1; }
timeout -k 10 300 python bench.py --config c4 --T 500 > $O/c4_T500.log 2>$O/c4_T500.err || { tail -20 $O/c4_T500.err; exit 1; }
echo ALLOK
