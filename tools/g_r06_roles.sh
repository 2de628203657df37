#!/bin/bash
# GPU recipe (round 6): where the C2 step's time goes against the byte-movement ceiling of its own shape, one box --
# the shape probe (tools/probe/c2_shape_probe: read-only / write-only / split roles without arithmetic), then the C2
# line on this tree and on the role-ablation builds (INSITE_DEF_ROLES 1 = gram role alone, 2 = rollout role alone).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_roles${TAG}
mkdir -p $O
AB=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
show() { python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline',{})
print(sys.argv[2], round(d['ms_per_step'],5), round(r.get('avg_launch_ms',0),5), round(r.get('frac',0),4))" $1 $2; }
if [ -n "$TESTS" ]; then
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
fi
if [ -z "$NOPROBE" ]; then timeout -k 10 60 ./tools/probe/c2_shape_probe 100032 200 1 > $O/probe_c2.json || exit 1; fi
[ -z "$NOPROBE" ] && cat $O/probe_c2.json
for rep in $(seq 1 ${REPS:-2}); do
  for v in default ${VARS:-gramonly rollonly}; do
    if [ "$v" = default ]; then L=""; else L="$AB/libinsite_hip_$v.so"; fi
    INSITE_LIB_OVERRIDE=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --no-north-star --no-c3-block --steps 100 > $O/c2_${v}_$rep.jsonl 2> $O/c2_${v}_$rep.err || { echo "c2 $v failed"; tail -5 $O/c2_${v}_$rep.err; exit 1; }
    show $O/c2_${v}_$rep.jsonl c2_$v
  done
done
echo RDONE
