#!/bin/bash
# RK45 flat loop vs per-interval (A/B), parity tests, C5 bench + rocprof stats
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_rk45.py tests/test_gpu_plugin.py -x -q --timeout 200 --timeout-method thread > $O/rk45_tests.log 2>&1 || { tail -40 $O/rk45_tests.log; exit 1; }
tail -2 $O/rk45_tests.log
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/c5_flat.log 2>$O/c5_flat.err || { tail -20 $O/c5_flat.err; exit 1; }
INSITE_LIB_OVERRIDE=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate/libinsite_hip_RK45PI.so timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/c5_pi.log 2>$O/c5_pi.err || { tail -20 $O/c5_pi.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --config c5 --no-cpu-baseline > $O/c5_prof.log 2>&1 || { tail -20 $O/c5_prof.log; exit 1; }
echo ALLOK
