#!/bin/bash
# C3 Gram tail: 4x4x4 f64 MFMA (default) vs the padded 16x16 tile (MSTAIL0); parity first
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_multistate.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t_mstail.log 2>&1 || { tail -30 gpurun_out/t_mstail.log; exit 1; }
tail -1 gpurun_out/t_mstail.log
A=ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
for v in default MSTAIL0 default MSTAIL0; do
  if [ $v = default ]; then unset INSITE_LIB_OVERRIDE; else export INSITE_LIB_OVERRIDE=$A/libinsite_hip_$v.so; fi
  timeout -k 10 240 python bench.py --config c3 --steps 3 --warmup 1 > gpurun_out/c3_$v.log 2>&1 || { tail -20 gpurun_out/c3_$v.log; exit 1; }
  tail -1 gpurun_out/c3_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config']['support_equals_truth'])"
done
