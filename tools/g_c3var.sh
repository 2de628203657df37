#!/bin/bash
# C3 bench: default build + profiling-only ablation variants (gram time per variant)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-c3var}
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
mkdir -p $O
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > $O/c3.log 2>$O/c3.err || { tail -20 $O/c3.err; exit 1; }
for v in ${VARIANTS}; do INSITE_LIB_OVERRIDE=$A/libinsite_hip_$v.so timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > $O/c3_$v.log 2>$O/c3_$v.err || { tail -20 $O/c3_$v.err; exit 1; }; done
for f in $O/c3*.log; do python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[1], round(d['ms_per_step'],3), round(r['avg_launch_ms'],3), round(r['frac'],3))" $f; done
echo ALLOK
