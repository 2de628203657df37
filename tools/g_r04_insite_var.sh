set -o pipefail
cd $GRAFT_REPO_ROOT
L=$PWD/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_insite.py tests/test_gpu_refine_general.py tests/test_gpu_reference.py > gpurun_out/r04_t4.txt 2>&1 || exit 1
for v in ${VARIANTS:-default NOWIN}; do
  if [ $v = default ]; then unset INSITE_LIB_OVERRIDE; else export INSITE_LIB_OVERRIDE=$L/libinsite_hip_$v.so; fi
  echo "== $v" >> gpurun_out/r04_insite_var3.txt
  timeout -k 10 300 python bench.py --config insite --no-cpu-baseline --steps 10 --warmup 3 >> gpurun_out/r04_insite_var3.txt 2>> gpurun_out/r04_insite_var.err || exit 1
done
unset INSITE_LIB_OVERRIDE
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04_prof_insite2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config insite --no-cpu-baseline --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/r04_prof_insite2.log 2>&1
