set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_seg
mkdir -p $O
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
for rep in 1 2; do
for var in base KC8W3 KC16W2; do
  if [ $var = base ]; then E="X=1"; else E="INSITE_LIB_OVERRIDE=$A/libinsite_hip_$var.so"; fi
  timeout -k 10 200 env $E python bench.py --config f4 --no-cpu-baseline --steps 20 --warmup 5 > $O/f4_${var}_$rep.jsonl 2>/dev/null || exit 1
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],4), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_ms'],4))" $O/f4_${var}_$rep.jsonl $var
done
done
