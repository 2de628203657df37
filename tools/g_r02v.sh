#!/bin/bash
# fused step kernel with two patients per rollout lane: tests, role probe, split sweep (A/B vs PPL 1)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02v}
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/fused_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
cat $O/probe.log
for v in default ${VARIANTS:-STEPPPL1}; do
  for gb in ${SPLITS:-256 288 320 352 384}; do
    if [ $v = default ]; then unset INSITE_LIB_OVERRIDE; else export INSITE_LIB_OVERRIDE=$A/libinsite_hip_$v.so; fi
    timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --gram-blocks $gb --steps 50 > $O/${v}_$gb.log 2>$O/${v}_$gb.err || { tail -20 $O/${v}_$gb.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${v}_$gb.log'));print('$v gb',$gb,'ms',round(d['ms_per_step'],5),'ev',round(d['roofline']['avg_launch_ms'],5),'frac',round(d['roofline']['frac'],3))"
  done
done
unset INSITE_LIB_OVERRIDE
timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --mode pipeline --steps 50 > $O/pipe.log 2>$O/pipe.err || { tail -20 $O/pipe.err; exit 1; }
python -c "import json;d=json.load(open('$O/pipe.log'));print('pipeline ms',round(d['ms_per_step'],5))"
echo ALLOK
