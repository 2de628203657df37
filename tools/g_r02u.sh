#!/bin/bash
# fused step kernel: split sweep only (bench), a few repeats of the best candidates
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02u}
mkdir -p $O
for gb in ${SPLITS:-288 320 352 384 416 448 480}; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --gram-blocks $gb --steps 50 > $O/fused_$gb.log 2>$O/fused_$gb.err || { tail -20 $O/fused_$gb.err; exit 1; }
  python -c "import json;d=json.load(open('$O/fused_$gb.log'));print('gb',$gb,'ms',round(d['ms_per_step'],5),'ev',round(d['roofline']['avg_launch_ms'],5),'frac',round(d['roofline']['frac'],3))"
done
for m in ${MODES:-pipeline}; do
timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --mode $m --steps 50 > $O/$m.log 2>$O/$m.err || { tail -20 $O/$m.err; exit 1; }
python -c "import json;d=json.load(open('$O/$m.log'));print('$m ms',round(d['ms_per_step'],5))"
done
echo ALLOK
