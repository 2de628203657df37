#!/bin/bash
# GPU recipe (round 6, final): PART=a -- every GPU test, smoke(), the default bench line (C2 + north_star_step + c3
# blocks), rocprofv3 kernel stats of the same command; PART=b -- the secondary lines with
# their parity blocks, then (TRAFFIC) the PMC traffic passes of the named configs.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_final${TAG}
mkdir -p $O
if [ "${PART:-a}" = a ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/test_gpu_all.txt 2>&1 || { tail -40 $O/test_gpu_all.txt; exit 1; }
tail -2 $O/test_gpu_all.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench_default.jsonl 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 - $O/bench_default.jsonl <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
p = d.get("parity", {})
print("default", round(d["ms_per_step"], 5), "frac", round(d["roofline"]["frac"], 4), p.get("support_equal"), p.get("coef_linf"), p.get("y_rmse"))
ns = d.get("north_star_step", {})
print("ns", ns.get("error") or (round(ns["ms_per_step"], 4), round(ns["roofline"]["frac"], 4), {k: ns.get("parity", {}).get(k) for k in ("support_equal", "coef_linf", "y_rmse", "oracle_seconds")}))
c3 = d.get("c3", {})
print("c3", c3.get("error") or (round(c3["ms_per_step"], 3), round(c3["roofline"]["frac"], 4), {k: c3.get("parity", {}).get(k) for k in ("support_equal", "coef_linf", "gram_max_rel_sampled_tiles")}))
print("nsr", d.get("north_star_rollout", {}).get("frac_of_8TBps"))
PY
cd /tmp && export TMPDIR=/tmp
# the default line's own command (its C2 launches are step_deferred_kernel<.., 0>, the north-star block's the claimed
# instantiation <.., 1>: two rows of one profile, from the same process layout as the line)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_default -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-parity > $GRAFT_REPO_ROOT/$O/prof_default.jsonl 2> $GRAFT_REPO_ROOT/$O/prof_default.log && echo PROF default ok
else
for c in ${LINES:-c3 c4 c5 f4 insite insite4}; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.jsonl 2> $O/bench_$c.err || { echo "bench $c failed"; tail -5 $O/bench_$c.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); cb=d.get('cpu_baseline') or {}
print(sys.argv[2], round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],4), 'cpu', round(cb.get('value',0),1), cb.get('cores'))" $O/bench_$c.jsonl $c
done
if [ -n "$TRAFFIC" ]; then
CONFIGS="$TRAFFIC" OUT=r06_final${TAG}/traffic PMC_LIMIT=240 bash tools/g_traffic.sh || exit 1
fi
fi
