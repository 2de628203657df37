#!/bin/bash
# stage-evaluated RK4 / Euler-5 rollout (ablation build: the reference's stage arithmetic per step instead of
# the interval map) vs the default: parity vs the oracle, C2 / north-star / C4 rollout timings
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02al}
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
mkdir -p $O
for v in default STAGEWISE; do
  if [ $v = default ]; then unset INSITE_LIB_OVERRIDE; else export INSITE_LIB_OVERRIDE=$A/libinsite_hip_$v.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_fused.py -x -q --timeout 200 --timeout-method thread -k "rollout or north or fused" > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
  echo "$v $(tail -1 $O/tests_$v.log)"
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-fused --isolated --steps 50 > $O/${v}_c2.log 2>$O/${v}_c2.err || { tail -5 $O/${v}_c2.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${v}_c2.log'));print('$v c2 ms',round(d['ms_per_step'],5),'iso',d['isolated'],'north',round(d['north_star_rollout']['avg_launch_ms'],4),round(d['north_star_rollout']['frac_of_8TBps'],3))"
  timeout -k 10 300 python bench.py --config c4 --no-cpu-baseline > $O/${v}_c4.log 2>$O/${v}_c4.err || { tail -5 $O/${v}_c4.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/${v}_c4.log').read().splitlines()[-1]);print('$v c4 ms',round(d['ms_per_step'],4),'roll',round(d['roofline']['avg_launch_ms'],4),round(d['roofline']['frac'],3))"
done
echo ALLOK
