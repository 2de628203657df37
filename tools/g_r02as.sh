#!/bin/bash
# per-patient fit kernel sized for 2 (default) / 3 / 4 waves per SIMD: C4 line (T = 60)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02as}
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
mkdir -p $O
for v in default PPW3 PPW4; do
  if [ $v = default ]; then unset INSITE_LIB_OVERRIDE; else export INSITE_LIB_OVERRIDE=$A/libinsite_hip_$v.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_moments.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "patient or one_pass" > $O/tests_$v.log 2>&1 || { tail -20 $O/tests_$v.log; exit 1; }
  echo "$v $(tail -1 $O/tests_$v.log)"
  for r in 1 2; do
  timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $O/${v}_c4_$r.log 2>$O/err || { tail -5 $O/err; exit 1; }
  python -c "import json;d=json.loads(open('$O/${v}_c4_$r.log').read().splitlines()[-1]);print('$v c4 ms',round(d['ms_per_step'],4),'pp',round(d['per_patient_fit']['avg_ms'],4))"
  done
done
echo ALLOK
