#!/bin/bash
# C3 moment cover: multistate GPU tests + the C3 config-scale test, then the C3 bench line on the default build
# and on the listed variant libraries (VARIANTS), gram_ms4_kernel time per variant.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-c3cover}
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
mkdir -p $O
if [ -z "$NOTEST" ]; then
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_multistate.py \
  tests/test_gpu_config_scale.py -k "gram_ms or c3 or stlsq_wave" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
fi
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > $O/c3.log 2>$O/c3.err || { tail -20 $O/c3.err; exit 1; }
for v in ${VARIANTS}; do INSITE_LIB_OVERRIDE=$A/libinsite_hip_$v.so timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-parity > $O/c3_$v.log 2>$O/c3_$v.err || { tail -20 $O/c3_$v.err; exit 1; }; done
for f in $O/c3*.log; do python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[1], round(d['ms_per_step'],3), round(r['avg_launch_ms'],3), round(r['frac'],3), {k: d.get('parity',{}).get(k) for k in ('gram_max_rel_sampled_tiles','support_equal','coef_linf')})" $f; done
echo ALLOK
