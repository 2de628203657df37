#!/bin/bash
# fused default: gram-block split sweep at the driver's 20 steps, 3 rounds
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02aw}
mkdir -p $O
for r in 1 2 3; do
  for gb in 0 256 288 336 368; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --gram-blocks $gb > $O/f${gb}_$r.log 2>$O/err || { tail -5 $O/err; exit 1; }
    python -c "import json;d=json.load(open('$O/f${gb}_$r.log'));print('gb $gb r $r',round(d['ms_per_step'],5),round(d['roofline']['avg_launch_ms'],5))"
  done
done
echo ALLOK
