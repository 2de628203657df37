#!/bin/bash
# F4 / C4 lines with their multi-core CPU baselines
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02ar}
mkdir -p $O
run() { n=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/$n.log 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/$n.log').read().splitlines()[-1]);c=d.get('cpu_baseline') or {};print('$n ms',round(d['ms_per_step'],4),'cpu',c.get('value'),c.get('cores'),c.get('sample'))"; }
run f4 --config f4
run c4_T60 --config c4
echo ALLOK
