#!/bin/bash
# default bench (K = 8) three times as the driver runs it, then the 2-rank rehearsal
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02ao}
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$r.log 2>$O/err || { tail -5 $O/err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$r.log').read().splitlines()[-1]);print('r $r ms',round(d['ms_per_step'],5),'roof',round(d['roofline']['frac'],3),'agg',round(d['step_aggregate']['frac'],3),d['config']['discovered_support'])"
done
OUT=r02ao_rh bash tools/g_r02ae.sh
