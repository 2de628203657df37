set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_steps
timeout -k 10 400 python -u -m pytest tests/test_gpu_deferred.py tests/test_gpu_fused.py tests/test_gpu_dist.py -x -q > gpurun_out/r04_steps/tests.txt 2>&1 || { tail -30 gpurun_out/r04_steps/tests.txt; exit 1; }
tail -1 gpurun_out/r04_steps/tests.txt
V=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate/libinsite_hip_UNITS.so
for rep in 1 2 3; do
  for var in steps units; do
    if [ $var = units ]; then E="INSITE_LIB_OVERRIDE=$V"; else E="X=1"; fi
    timeout -k 10 120 env $E python bench.py --no-cpu-baseline --no-north-star --steps 100 --warmup 10 > gpurun_out/r04_steps/${var}_$rep.jsonl 2>/dev/null || exit 1
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],5), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_ms'],5))" gpurun_out/r04_steps/${var}_$rep.jsonl $var
  done
done
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 150 rocprofv3 --pmc $C -d $GRAFT_REPO_ROOT/gpurun_out/r04_steps/pmc_$C -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-north-star --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r04_steps/pmc_$C.log 2>&1 || exit 1
done
echo PMC ok
