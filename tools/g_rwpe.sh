set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
A=ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
for v in ${RWPE_VARIANTS:-default RWPE1 RWPE3}; do
  if [ $v = default ]; then unset INSITE_LIB_OVERRIDE; else export INSITE_LIB_OVERRIDE=$PWD/$A/libinsite_hip_$v.so; fi
  timeout -k 10 200 python bench.py --config insite --no-cpu-baseline > gpurun_out/rw_$v.log 2>&1
  echo $v $(tail -1 gpurun_out/rw_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['insite']['converged'], d['insite']['mean_bfgs_iterations'])")
done
unset INSITE_LIB_OVERRIDE
timeout -k 10 300 python -u -m pytest tests/test_gpu_insite.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_insite.log 2>&1; tail -1 gpurun_out/t_insite.log
