#!/bin/bash
# gram time tile / ring depth variants (GT8: 8-step tiles, D = tiles in the register ring): parity of the
# C2 discovery paths under each variant, then C2 bench in pipeline / fused / seq modes
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02w}
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
mkdir -p $O
for v in default ${VARIANTS:-GT8D4 GT8D3 GT8D5}; do
  if [ $v = default ]; then unset INSITE_LIB_OVERRIDE; else export INSITE_LIB_OVERRIDE=$A/libinsite_hip_$v.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_reference.py -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
  echo "$v $(tail -1 $O/tests_$v.log)"
  for m in pipeline fused seq; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --mode $m --steps 50 --isolated > $O/${v}_$m.log 2>$O/${v}_$m.err || { tail -20 $O/${v}_$m.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${v}_$m.log'));print('$v $m ms',round(d['ms_per_step'],5),'iso',{k:round(x,4) for k,x in d.get('isolated',{}).items()})"
  done
done
echo ALLOK
