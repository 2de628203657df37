set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_lnt
timeout -k 10 400 python -u -m pytest tests/test_gpu_deferred.py tests/test_gpu_fused.py tests/test_gpu_dist.py -x -q > gpurun_out/r04_lnt/tests.txt 2>&1 || { tail -30 gpurun_out/r04_lnt/tests.txt; exit 1; }
tail -1 gpurun_out/r04_lnt/tests.txt
V=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate/libinsite_hip_LNT.so
for rep in 1 2 3; do
  for var in base lnt; do
    if [ $var = lnt ]; then E="INSITE_LIB_OVERRIDE=$V"; else E="X=1"; fi
    timeout -k 10 120 env $E python bench.py --no-cpu-baseline --no-north-star --steps 100 --warmup 10 > gpurun_out/r04_lnt/${var}_$rep.jsonl 2>/dev/null || exit 1
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],5), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_ms'],5))" gpurun_out/r04_lnt/${var}_$rep.jsonl $var
  done
done
