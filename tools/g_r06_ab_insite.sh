#!/bin/bash
# GPU recipe (round 6): INSITE M = 3 line (bench.py --config insite, nfev order) across lib/ablate builds, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_abins${TAG}
mkdir -p $O
AB=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
for rep in 1 2; do
  for v in default ${VARS}; do
    if [ "$v" = default ]; then L=""; else L="$AB/libinsite_hip_$v.so"; fi
    INSITE_LIB_OVERRIDE=$L timeout -k 10 400 python bench.py --config ${CFG:-insite} --no-cpu-baseline --no-parity > $O/${v}_$rep.jsonl 2> $O/${v}_$rep.err || { echo "$v failed"; tail -5 $O/${v}_$rep.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline',{})
print(sys.argv[2], round(d['ms_per_step'],5), round(r.get('avg_launch_ms',0) or 0,5))" $O/${v}_$rep.jsonl $v
  done
done
echo ABDONE
