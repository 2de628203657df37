#!/bin/bash
# time-major int8-arm rollout (F4: 4 arms, 1M x 60): patients per lane 2 (default) vs 1 vs 4
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02ap}
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
mkdir -p $O
for v in default PPL1 PPL4; do
  if [ $v = default ]; then unset INSITE_LIB_OVERRIDE; else export INSITE_LIB_OVERRIDE=$A/libinsite_hip_$v.so; fi
  timeout -k 10 300 python bench.py --config f4 --no-cpu-baseline > $O/${v}_f4.log 2>$O/err || { tail -5 $O/err; exit 1; }
  python -c "import json;d=json.loads(open('$O/${v}_f4.log').read().splitlines()[-1]);print('$v f4 ms',round(d['ms_per_step'],4),'roll',d['rollout'])"
done
echo ALLOK
