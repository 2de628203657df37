set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
A=ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
for v in ${RA_VARIANTS:-default RW8_2 RREG8}; do
  if [ $v = default ]; then unset INSITE_LIB_OVERRIDE; else export INSITE_LIB_OVERRIDE=$PWD/$A/libinsite_hip_$v.so; fi
  echo $v $(timeout -k 10 300 python tools/refine_arms_bench.py 2> gpurun_out/ra_$v.err)
done
