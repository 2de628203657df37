#!/bin/bash
# GPU recipe (round 6): the INSITE lines' evaluation-count binning key resolution (INSITE_NFEV_KEY), interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_nfkey${TAG}
mkdir -p $O
for rep in 1 2; do
  for k in 64x16 32x32; do
    for c in insite insite4; do
      INSITE_NFEV_KEY=$k timeout -k 10 400 python bench.py --config $c --no-cpu-baseline --no-parity > $O/${c}_${k}_$rep.jsonl 2> $O/${c}_${k}_$rep.err || { echo "$c $k failed"; tail -5 $O/${c}_${k}_$rep.err; exit 1; }
      python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); i=d.get('insite',{}); m=d.get('models',{})
print(sys.argv[2], round(d['ms_per_step'],4), round(i.get('divergence',{}).get('ratio',0),4) if i else {k:(round(v['ms_per_step'],3), round(v['wave_divergence']['max_over_mean_evaluations'],3)) for k,v in m.items()})" $O/${c}_${k}_$rep.jsonl ${c}_$k
    done
  done
done
echo KDONE
