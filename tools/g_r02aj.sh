#!/bin/bash
# cross-item tile prefetch in the time-major gram: parity, C4 / C2 / fused lines
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02aj}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/$n.log').read().splitlines()[-1]);print('$n ms',round(d['ms_per_step'],4),'disc',(d.get('discovery') or {}).get('avg_ms'),'roof',d['roofline'].get('frac'))"; }
run c4_T60 --config c4 --no-cpu-baseline
run c4_T500 --config c4 --T 500 --no-cpu-baseline
run c2 --no-cpu-baseline --no-north-star --no-fused
run fused --no-cpu-baseline --no-north-star --mode fused
run f4 --config f4 --no-cpu-baseline
echo ALLOK
