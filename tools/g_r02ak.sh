#!/bin/bash
# same-box A/B: pipeline vs fused (several splits), 3 rounds interleaved
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02ak}
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --no-fused --steps 100 > $O/pipe_$r.log 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$O/pipe_$r.log'));print('pipe $r',round(d['ms_per_step'],5))"
  for gb in 0 256 288 352; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --mode fused --gram-blocks $gb --steps 100 > $O/f${gb}_$r.log 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$O/f${gb}_$r.log'));print('fused $gb $r',round(d['ms_per_step'],5),round(d['roofline']['avg_launch_ms'],5),round(d['roofline']['frac'],3))"
  done
done
echo ALLOK
