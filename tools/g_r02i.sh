#!/bin/bash
# C5 A/B: binned vs identity order, cached vs nontemporal patient-major stores
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02i}
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_rk45.py -x -q --timeout 200 --timeout-method thread > $O/rk45_tests.log 2>&1 || { tail -40 $O/rk45_tests.log; exit 1; }
tail -1 $O/rk45_tests.log
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/c5.log 2>$O/c5.err || { tail -20 $O/c5.err; exit 1; }
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --rk45-identity-order > $O/c5_id.log 2>$O/c5_id.err || { tail -20 $O/c5_id.err; exit 1; }
INSITE_LIB_OVERRIDE=$A/libinsite_hip_RKPMNT.so timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/c5_nt.log 2>$O/c5_nt.err || { tail -20 $O/c5_nt.err; exit 1; }
INSITE_LIB_OVERRIDE=$A/libinsite_hip_RKPMNT.so timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --rk45-identity-order > $O/c5_nt_id.log 2>$O/c5_nt_id.err || { tail -20 $O/c5_nt_id.err; exit 1; }
echo ALLOK
