#!/bin/bash
# GPU recipe (round 6): INSITE M = 3 line, lanes binned by seq_len vs by seq_len + the previous step's evaluation
# counts (--insite-order), interleaved on one box; the refinement GPU tests first.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_insite${TAG}
mkdir -p $O
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_insite.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
fi
for rep in $(seq 1 ${REPS:-2}); do
  for o in seq_len nfev; do
    timeout -k 10 400 python bench.py --config insite --no-cpu-baseline ${EXTRA:-} --insite-order $o > $O/insite_${o}_$rep.jsonl 2> $O/insite_${o}_$rep.err || { echo "insite $o failed"; tail -5 $O/insite_${o}_$rep.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline',{}); i=d.get('insite',{}); p=d.get('parity') or {}
print(sys.argv[2], round(d['ms_per_step'],4), 'kern', round(r.get('avg_launch_ms',0) or 0,4), 'div', round(i.get('divergence',{}).get('ratio',0),3), 'wmax', round(i.get('divergence',{}).get('mean_wave_max_nfev',0),2), 'eq', i.get('plan_equals_eager'), p.get('status_equal_frac'))" $O/insite_${o}_$rep.jsonl $o
  done
done
echo IDONE
