# GPU recipe (round 5): the dense 4-arm INSITE kernels -- bitwise / oracle tests, then the insite4 line.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_coop${TAG}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_insite.py tests/test_gpu_refine_general.py tests/test_gpu_reference_segments.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
timeout -k 10 500 python bench.py --config insite4 --no-cpu-baseline ${BARGS} > $O/bench_insite4.jsonl 2> $O/bench_insite4.err || { tail -5 $O/bench_insite4.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k,v in d['models'].items(): print(k, round(v['ms_per_step'],3), 'kern', round(v['kernel_ms'],3), v['kernel'], {a: v.get('parity',{}).get(a) for a in ('status_equal_frac','coef_linf','pred_rmse')})" $O/bench_insite4.jsonl
