set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_lines
for c in c3 c4 c5 f4 insite insite4; do
  timeout -k 10 400 python bench.py --config $c > gpurun_out/r04_lines/bench_$c.jsonl 2> gpurun_out/r04_lines/bench_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/r04_lines/bench_$c.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); cb=d.get('cpu_baseline') or {}
print(sys.argv[2], round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],4), 'cpu', round(cb.get('value',0),1), cb.get('cores'))" gpurun_out/r04_lines/bench_$c.jsonl $c
done
CONFIGS="insite:--config insite;insite4:--config insite4" OUT=r04_traffic_insite PMC_LIMIT=240 bash tools/g_traffic.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04_lines/prof_c2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py > $GRAFT_REPO_ROOT/gpurun_out/r04_lines/prof_c2.log 2>&1 && echo PROF ok
