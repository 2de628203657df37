#!/bin/bash
# RK45 flat loop v3 (one fifth root per iteration, register queue): parity tests, C5 bench, rocprof stats,
# one SQ PMC pass (issue vs wait split)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02d}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_rk45.py tests/test_gpu_plugin.py -x -q --timeout 200 --timeout-method thread > $O/rk45_tests.log 2>&1 || { tail -40 $O/rk45_tests.log; exit 1; }
tail -2 $O/rk45_tests.log
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/c5.log 2>$O/c5.err || { tail -20 $O/c5.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --config c5 --no-cpu-baseline --steps 5 --warmup 2 > $O/c5_prof.log 2>&1 || { tail -20 $O/c5_prof.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $O/pmc -o pmc --output-format csv -- python3 bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > $O/c5_pmc.log 2>&1 || { tail -20 $O/c5_pmc.log; exit 1; }
echo ALLOK
