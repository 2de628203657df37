set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_cf
mkdir -p $O
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
timeout -k 10 600 python -u -m pytest tests/test_gpu_insite.py tests/test_gpu_refine_general.py tests/test_gpu_reference_segments.py tests/test_gpu_reference.py -x -q --timeout 300 > $O/tests.txt 2>&1; echo "tests rc $?"; tail -15 $O/tests.txt
for rep in 1 2; do
  for var in cf nocf cfw2; do
    case $var in cf) E="X=1";; nocf) E="INSITE_LIB_OVERRIDE=$A/libinsite_hip_NOCF.so";; cfw2) E="INSITE_LIB_OVERRIDE=$A/libinsite_hip_CFW2.so";; esac
    timeout -k 10 200 env $E python bench.py --config insite --no-cpu-baseline --steps 10 --warmup 2 > $O/insite_${var}_$rep.jsonl 2>/dev/null || exit 1
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['config'].get('mean_evaluations_per_refined_row', d.get('mean_evaluations_per_refined_row')))" $O/insite_${var}_$rep.jsonl $var
  done
done
for var in cf nocf; do
  case $var in cf) E="X=1";; nocf) E="INSITE_LIB_OVERRIDE=$A/libinsite_hip_NOCF.so";; esac
  timeout -k 10 400 env $E python bench.py --config insite4 --no-cpu-baseline --steps 3 --warmup 1 > $O/insite4_$var.jsonl 2>/dev/null || exit 1
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], {k:(round(v['ms_per_step'],2), round(v['kernel_ms'],2), round(v['mean_evaluations_per_refined_row'],3)) for k,v in d['models'].items()})" $O/insite4_$var.jsonl $var
done
