#!/bin/bash
# secondary configuration lines (C3, C4 T=60/500, C5, INSITE, F4) on the current tree + C5/F4 kernel stats
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02ad}
mkdir -p $O
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/$n.log').read().splitlines()[-1]);r=d.get('roofline') or {};print('$n ms',round(d['ms_per_step'],4),'frac',r.get('frac'))"; }
run f4 --config f4 --no-cpu-baseline
run c5 --config c5 --no-cpu-baseline
run c4_T60 --config c4 --no-cpu-baseline
run c4_T500 --config c4 --T 500 --no-cpu-baseline
run c3 --config c3 --no-cpu-baseline
run insite --config insite --no-cpu-baseline
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_f4 -o run --output-format csv -- python3 bench.py --config f4 --no-cpu-baseline --steps 5 --warmup 1 > $O/f4_prof.log 2>&1 || { tail -20 $O/f4_prof.log; exit 1; }
head -4 $O/prof_f4/run_kernel_stats.csv | cut -c1-200
echo ALLOK
