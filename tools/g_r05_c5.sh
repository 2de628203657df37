# GPU recipe (round 5): RK45 tests (C5 kernel vs the oracle, attempt counts) and the C5 line on the default build
# and on the listed variant libraries (VARIANTS).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_c5${TAG}
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rk45.py tests/test_gpu_config_scale.py -m gpu -x -q --timeout 300 --timeout-method thread -k "rk45 or c5" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2; do
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/c5_$rep.jsonl 2> $O/c5_$rep.err || { tail -5 $O/c5_$rep.err; exit 1; }
for v in ${VARIANTS}; do INSITE_LIB_OVERRIDE=$A/libinsite_hip_$v.so timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-parity > $O/c5_${v}_$rep.jsonl 2> $O/c5_${v}_$rep.err || { tail -5 $O/c5_${v}_$rep.err; exit 1; }; done
done
for f in $O/c5*.jsonl; do python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']
print(sys.argv[1], round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms'],4), (d.get('parity') or {}).get('attempts_equal_frac'))" $f; done
