set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_m6
mkdir -p $O
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
timeout -k 10 600 python -u -m pytest tests/test_gpu_insite.py tests/test_gpu_refine_general.py tests/test_gpu_reference_segments.py -x -q --timeout 300 > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2; do
for var in m6 nom6; do
  case $var in m6) E="X=1";; nom6) E="INSITE_LIB_OVERRIDE=$A/libinsite_hip_NOM6.so";; esac
  timeout -k 10 400 env $E python bench.py --config insite4 --no-cpu-baseline --steps 3 --warmup 1 > $O/insite4_${var}_$rep.jsonl 2>/dev/null || exit 1
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], {k:(round(v['ms_per_step'],2), round(v['kernel_ms'],2)) for k,v in d['models'].items()})" $O/insite4_${var}_$rep.jsonl $var
done
done
