#!/bin/bash
# occupancy-3 builds (gram + step kernel sized for 3 waves/SIMD: spills) vs default: kernels + C2 modes +
# fused split sweep; then the 2-rank rehearsal with the bucketed all-reduce
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02ag}
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
mkdir -p $O
for v in default ${VARIANTS:-WPE3 SWPE3}; do
  if [ $v = default ]; then unset INSITE_LIB_OVERRIDE; else export INSITE_LIB_OVERRIDE=$A/libinsite_hip_$v.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 200 --timeout-method thread > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
  echo "$v $(tail -1 $O/tests_$v.log)"
  for op in gram sindy_fit; do
    timeout -k 10 120 python tools/kbench.py --op $op --layout time --iters 50 > $O/${v}_kb_$op.json 2>/dev/null || exit 1
    echo "$v $op $(python -c "import json;print(round(json.load(open('$O/${v}_kb_$op.json'))['ms_per_call']*1e3,2))") us"
  done
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --no-fused --steps 50 > $O/${v}_pipe.log 2>$O/${v}_pipe.err || { tail -5 $O/${v}_pipe.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${v}_pipe.log'));print('$v pipeline ms',round(d['ms_per_step'],5))"
  for gb in 0 320 384 448 512; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --mode fused --gram-blocks $gb --steps 50 > $O/${v}_f$gb.log 2>$O/${v}_f$gb.err || { tail -5 $O/${v}_f$gb.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${v}_f$gb.log'));print('$v fused gb $gb ms',round(d['ms_per_step'],5),'frac',round(d['roofline']['frac'],3))"
  done
done
unset INSITE_LIB_OVERRIDE
OUT=r02af bash tools/g_r02ae.sh
