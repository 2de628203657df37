#!/bin/bash
# fused step from a HIP graph vs eager launches vs the pipeline, same box, 3 rounds
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02am}
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --no-fused --steps 100 > $O/pipe_$r.log 2>$O/err || { tail -5 $O/err; exit 1; }
  python -c "import json;d=json.load(open('$O/pipe_$r.log'));print('pipe $r',round(d['ms_per_step'],5))"
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --mode fused --steps 100 > $O/fe_$r.log 2>$O/err || { tail -5 $O/err; exit 1; }
  python -c "import json;d=json.load(open('$O/fe_$r.log'));print('fused eager $r',round(d['ms_per_step'],5),round(d['roofline']['avg_launch_ms'],5))"
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --mode fused --fused-graph --steps 100 > $O/fg_$r.log 2>$O/err || { tail -5 $O/err; exit 1; }
  python -c "import json;d=json.load(open('$O/fg_$r.log'));print('fused graph $r',round(d['ms_per_step'],5),round(d['roofline']['avg_launch_ms'],5),d['config']['discovered_support'])"
done
echo ALLOK
