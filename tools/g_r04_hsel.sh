set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_hsel
mkdir -p $O
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
timeout -k 10 600 python -u -m pytest $(grep -ln rk45 tests/test_gpu*.py) -x -q --timeout 300 > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2 3; do
for var in hsel nohsel; do
  case $var in hsel) E="X=1";; nohsel) E="INSITE_LIB_OVERRIDE=$A/libinsite_hip_NOHSEL.so";; esac
  timeout -k 10 200 env $E python bench.py --config c5 --no-cpu-baseline --steps 20 --warmup 5 > $O/c5_${var}_$rep.jsonl 2>/dev/null || exit 1
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['rk45']['mean_attempts_per_patient'])" $O/c5_${var}_$rep.jsonl $var
done
done
