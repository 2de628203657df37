set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
A=ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
for v in ${KWPE_VARIANTS:-default KWPE5 KWPE6 KWPE8}; do
  if [ $v = default ]; then unset INSITE_LIB_OVERRIDE; else export INSITE_LIB_OVERRIDE=$PWD/$A/libinsite_hip_$v.so; fi
  timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline > gpurun_out/kw_$v.log 2>&1
  echo $v $(tail -1 gpurun_out/kw_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['rk45']['mean_attempts_per_patient'])")
done
