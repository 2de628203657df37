#!/bin/bash
# GPU recipe (round 6): is the north-star line's first-allocation slowness a clock ramp or the allocation? (a soak of
# ~2 s of launches on the first allocation, then its third timing); and the C2 line at a ~1.5 s warmup.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_g${TAG}
mkdir -p $O
timeout -k 10 300 python tools/ns_variance.py --soak 1200 > $O/nsvar_soak.json 2> $O/nsvar_soak.err || { tail -5 $O/nsvar_soak.err; exit 1; }
cat $O/nsvar_soak.json
show() { python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline',{})
print(sys.argv[2], round(d['ms_per_step'],5), round(r.get('avg_launch_ms',0),5), round(r.get('frac',0),4))" $1 $2; }
for w in 5 20000 5 20000; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --no-north-star --no-c3-block --warmup $w --steps 100 > $O/c2_w$w.jsonl 2> $O/c2_w$w.err || { tail -5 $O/c2_w$w.err; exit 1; }
  show $O/c2_w$w.jsonl c2_warmup_$w
done
echo GDONE
