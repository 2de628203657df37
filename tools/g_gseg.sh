cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && : > gpurun_out/gseg.log
A=ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
timeout -k 10 120 python tools/kbench.py --op gram_seg --patients 1000000 --T 60 --iters 20 >> gpurun_out/gseg.log 2>&1 || exit 1
for v in SEGKC4 SEGKC16 SEGNOPF SEGKC16NOPF; do
  INSITE_LIB_OVERRIDE=$A/libinsite_hip_$v.so timeout -k 10 120 python tools/kbench.py --op gram_seg --patients 1000000 --T 60 --iters 20 >> gpurun_out/gseg.log 2>&1 || exit 1
done
timeout -k 10 120 python tools/kbench.py --op gram_seg --patients 1000000 --T 500 --iters 10 >> gpurun_out/gseg.log 2>&1
cat gpurun_out/gseg.log | grep ms_per_call
