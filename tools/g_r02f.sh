#!/bin/bash
# RK45 v4 (LDS time window): parity tests, C5 bench for the default build and the window/occupancy variants
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02f}
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_rk45.py tests/test_gpu_plugin.py -x -q --timeout 200 --timeout-method thread > $O/rk45_tests.log 2>&1 || { tail -40 $O/rk45_tests.log; exit 1; }
tail -2 $O/rk45_tests.log
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/c5.log 2>$O/c5.err || { tail -20 $O/c5.err; exit 1; }
for v in ${VARIANTS}; do
  INSITE_LIB_OVERRIDE=$A/libinsite_hip_$v.so timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/c5_$v.log 2>$O/c5_$v.err || { tail -20 $O/c5_$v.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --config c5 --no-cpu-baseline --steps 5 --warmup 2 > $O/c5_prof.log 2>&1 || { tail -20 $O/c5_prof.log; exit 1; }
echo ALLOK
