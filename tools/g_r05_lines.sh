# GPU recipe (round 5): the new bench-size INSITE parity test, then every secondary bench line with its oracle
# parity block.  usage: LINES="insite c5 ..." TAG=v1 bash tools/g_r05_lines.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_lines${TAG}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
  tail -2 $O/tests.txt
fi
for c in ${LINES:-insite insite4 c5 c4 c3 f4}; do
  timeout -k 10 500 python bench.py --config $c > $O/bench_$c.jsonl 2> $O/bench_$c.err || { echo "bench $c failed"; tail -5 $O/bench_$c.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); cb=d.get('cpu_baseline') or {}
p={k: v for k, v in (d.get('parity') or {}).items() if k not in ('oracle','cohort','tolerances')}
print(sys.argv[2], round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],4), 'cpu', round(cb.get('value',0),1), cb.get('cores'), 'parity', p)" $O/bench_$c.jsonl $c
done
