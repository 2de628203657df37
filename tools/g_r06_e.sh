#!/bin/bash
# GPU recipe (round 6): the north-star line with a claimed ROLLOUT tail as well (INSITE_DEF_RSTATIC / RCHUNK variant
# builds, the per-XCD heads at workspace offset 2 KiB) against this tree (claimed gram tail only) and nodyn, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_e${TAG}
mkdir -p $O
AB=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
show() { python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline',{}); p=d.get('parity') or {}
print(sys.argv[2], round(d['ms_per_step'],5), round(r.get('avg_launch_ms',0),5), round(r.get('frac',0),4), p.get('support_equal'), p.get('coef_linf'))" $1 $2; }
for rep in 1 2; do
  for v in default ${NSVARS:-nodyn rs800c16 rs900c16 rs800c8}; do
    if [ "$v" = default ]; then L=""; else L="$AB/libinsite_hip_$v.so"; fi
    INSITE_LIB_OVERRIDE=$L timeout -k 10 300 python bench.py --config ns --no-parity --ns-steps 20 > $O/ns_${v}_$rep.jsonl 2> $O/ns_${v}_$rep.err || { echo "ns $v failed"; tail -5 $O/ns_${v}_$rep.err; exit 1; }
    show $O/ns_${v}_$rep.jsonl ns_$v
  done
done
if [ -n "$PARV" ]; then
  INSITE_LIB_OVERRIDE=$AB/libinsite_hip_$PARV.so timeout -k 10 300 python bench.py --config ns > $O/ns_${PARV}_parity.jsonl 2> $O/ns_${PARV}_parity.err || { tail -5 $O/ns_${PARV}_parity.err; exit 1; }
  show $O/ns_${PARV}_parity.jsonl ns_${PARV}_parity
fi
echo EDONE
