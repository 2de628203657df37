#!/bin/bash
# GPU recipe (round 6): north-star step line (bench.py --config ns, no parity) A/B across lib/ablate builds, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_nsab${TAG}
mkdir -p $O
AB=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
for rep in $(seq 1 ${REPS:-2}); do
  for v in default ${VARS}; do
    if [ "$v" = default ]; then L=""; else L="$AB/libinsite_hip_$v.so"; fi
    INSITE_LIB_OVERRIDE=$L timeout -k 10 300 python bench.py --config ns --no-parity --ns-steps 20 > $O/ns_${v}_$rep.jsonl 2> $O/ns_${v}_$rep.err || { echo "ns $v failed"; tail -5 $O/ns_${v}_$rep.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline',{})
print(sys.argv[2], round(d['ms_per_step'],5), round(r.get('avg_launch_ms',0),5), round(r.get('frac',0),4))" $O/ns_${v}_$rep.jsonl ns_$v
  done
done
echo NSDONE
