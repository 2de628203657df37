#!/bin/bash
# pipeline: STLSQ in the gram tail (discovery stream) vs its own launch on the rollout stream; 3 repeats each
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02ac}
mkdir -p $O
for r in 1 2 3; do
for st in discovery rollout; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --no-fused --stlsq-stream $st --steps 100 > $O/${st}_$r.log 2>$O/${st}_$r.err || { tail -20 $O/${st}_$r.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${st}_$r.log'));print('$st $r ms',round(d['ms_per_step'],5),'roll',round(d['roofline']['avg_launch_ms'],4),'disc',round(d['discovery']['avg_ms'],4),d['config']['discovered_support'])"
done
done
echo ALLOK
