#!/bin/bash
# GPU recipe (round 6): north-star step line across gram-block counts (bench.py --config ns --gram-blocks), one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_nsgb${TAG}
mkdir -p $O
for rep in 1 2; do
for gb in ${GB:-0 224 288 320}; do
  timeout -k 10 300 python bench.py --config ns --no-parity --ns-steps 20 --gram-blocks $gb > $O/ns_gb${gb}_$rep.jsonl 2> $O/ns_gb${gb}_$rep.err || { echo "ns gb $gb failed"; tail -5 $O/ns_gb${gb}_$rep.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline',{})
print(sys.argv[2], round(d['ms_per_step'],5), round(r.get('avg_launch_ms',0),5), round(r.get('frac',0),4))" $O/ns_gb${gb}_$rep.jsonl ns_gb$gb
done
done
echo GBDONE
