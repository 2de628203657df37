set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_lines2
mkdir -p $O
for c in c3 c4 f4; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.jsonl 2> $O/bench_$c.err || { echo "bench $c failed"; tail -5 $O/bench_$c.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); cb=d.get('cpu_baseline') or {}
print(sys.argv[2], round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],4), 'cpu', round(cb.get('value',0),1), cb.get('cores'))" $O/bench_$c.jsonl $c
done
