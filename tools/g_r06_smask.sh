#!/bin/bash
# GPU recipe (round 6): the rollout's arm-mask forms A/B on one box, interleaved -- the north-star rollout alone
# (tools/nsr_ab.py, time- and tile-major bits) and the C2 step line, per library (VARS: lib/ablate builds).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_smask${TAG}
mkdir -p $O
AB=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
for rep in $(seq 1 ${REPS:-2}); do
  for v in default ${VARS:-smask0 smask2}; do
    if [ "$v" = default ]; then L=""; else L="$AB/libinsite_hip_$v.so"; fi
    INSITE_LIB_OVERRIDE=$L timeout -k 10 120 python tools/nsr_ab.py >> $O/nsr.jsonl || { echo "nsr $v failed"; exit 1; }
    if [ -z "$NOC2" ]; then
    INSITE_LIB_OVERRIDE=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --no-north-star --no-c3-block --steps 100 > $O/c2_${v}_$rep.jsonl 2> $O/c2_${v}_$rep.err || { echo "c2 $v failed"; tail -5 $O/c2_${v}_$rep.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline',{})
print(sys.argv[2], round(d['ms_per_step'],5), round(r.get('avg_launch_ms',0),5), round(r.get('frac',0),4))" $O/c2_${v}_$rep.jsonl c2_$v
    fi
  done
done
cat $O/nsr.jsonl
echo SDONE
# (GB: gram-block counts to sweep on the default library, the C2 line)
for gb in ${GB:-}; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --no-north-star --no-c3-block --steps 100 --gram-blocks $gb > $O/c2_gb${gb}.jsonl 2> $O/c2_gb${gb}.err || { echo "c2 gb $gb failed"; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline',{})
print(sys.argv[2], round(d['ms_per_step'],5), round(r.get('avg_launch_ms',0),5), round(r.get('frac',0),4))" $O/c2_gb${gb}.jsonl c2_gb$gb
done
