# GPU recipe (round 5): the INSITE row kernel's chunk-unrolled scan -- INSITE GPU tests (oracle parity, kernel-vs-
# kernel bitwise), then the insite line on the default build and on the loop-scan variant, twice each.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_scan${TAG}
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_insite.py tests/test_gpu_reference.py tests/test_gpu_reference_segments.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
show() { python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; p=d.get('parity') or {}
print(sys.argv[1], round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms'],4), p.get('status_equal_frac'), p.get('coef_linf_status_equal'))" $1; }
for rep in 1 2; do
for v in ${VARIANTS}; do INSITE_LIB_OVERRIDE=$A/libinsite_hip_$v.so timeout -k 10 400 python bench.py --config insite --no-cpu-baseline --no-parity > $O/insite_${v}_$rep.jsonl 2> $O/insite_${v}_$rep.err || { tail -5 $O/insite_${v}_$rep.err; exit 1; }; show $O/insite_${v}_$rep.jsonl; done
timeout -k 10 400 python bench.py --config insite --no-cpu-baseline > $O/insite_$rep.jsonl 2> $O/insite_$rep.err || { tail -5 $O/insite_$rep.err; exit 1; }
show $O/insite_$rep.jsonl
INSITE_LIB_OVERRIDE=$A/libinsite_hip_scanloop.so timeout -k 10 400 python bench.py --config insite --no-cpu-baseline --no-parity > $O/insite_loop_$rep.jsonl 2> $O/insite_loop_$rep.err || { tail -5 $O/insite_loop_$rep.err; exit 1; }
show $O/insite_loop_$rep.jsonl
done
