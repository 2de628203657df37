#!/bin/bash
# full GPU suite + every configuration's line on the current tree (round-end secondary evidence)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02aq}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/$n.log').read().splitlines()[-1]);r=d.get('roofline') or {};print('$n ms',round(d['ms_per_step'],4),'frac',r.get('frac'))"; }
run f4 --config f4
run c4_T60 --config c4
run c4_T500 --config c4 --T 500 --no-cpu-baseline
run c5 --config c5
run c3 --config c3
run insite --config insite
echo ALLOK
