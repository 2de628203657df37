#!/bin/bash
# C3: gram_ms4 (all 4x4x4 blocks) parity tests + bench, A/B vs the 16x16 form (MSV1) + kernel stats
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02s}
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_multistate.py -x -q --timeout 300 --timeout-method thread > $O/ms_tests.log 2>&1 || { tail -40 $O/ms_tests.log; exit 1; }
tail -1 $O/ms_tests.log
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > $O/c3.log 2>$O/c3.err || { tail -20 $O/c3.err; exit 1; }
for v in ${VARIANTS:-MSV1}; do INSITE_LIB_OVERRIDE=$A/libinsite_hip_$v.so timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > $O/c3_$v.log 2>$O/c3_$v.err || { tail -20 $O/c3_$v.err; exit 1; }; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --config c3 --no-cpu-baseline --steps 3 --warmup 1 > $O/c3_prof.log 2>&1 || { tail -20 $O/c3_prof.log; exit 1; }
echo ALLOK
