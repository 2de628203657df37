# GPU recipe (round 5): the RK45 binning -- RK45 / INSITE tests (the order feeds both), the C5 step gap probe, the
# C5 line twice at the default warmup and at 60 warmup steps.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_order${TAG}
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rk45.py tests/test_gpu_config_scale.py tests/test_gpu_insite.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 300 python -u tools/probe/c5_gap.py > $O/gap.txt 2>&1 || { tail -5 $O/gap.txt; exit 1; }
for rep in 1 2; do
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/c5_$rep.jsonl 2> $O/c5_$rep.err || { tail -5 $O/c5_$rep.err; exit 1; }
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-parity --warmup 60 > $O/c5_w60_$rep.jsonl 2> $O/c5_w60_$rep.err || { tail -5 $O/c5_w60_$rep.err; exit 1; }
done
for f in $O/c5*.jsonl; do python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[1], round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms'],4), (d.get('parity') or {}).get('attempts_equal_frac'))" $f; done
