#!/bin/bash
# fused step kernel: parity tests (fused + the rollout paths it shares), then the C2 bench sweep of the
# gram/rollout block split, then the pipeline mode for comparison
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02t}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_scale.py tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for gb in ${SPLITS:-0 128 160 196 224 256 288 320}; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --gram-blocks $gb > $O/fused_$gb.log 2>$O/fused_$gb.err || { tail -20 $O/fused_$gb.err; exit 1; }
  python -c "import json;d=json.load(open('$O/fused_$gb.log'));print('gb',$gb,'ms',round(d['ms_per_step'],5),'frac',round(d['roofline']['frac'],3),d['config']['discovered_support'])"
done
timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --mode pipeline > $O/pipe.log 2>$O/pipe.err || { tail -20 $O/pipe.err; exit 1; }
python -c "import json;d=json.load(open('$O/pipe.log'));print('pipeline ms',round(d['ms_per_step'],5))"
timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --isolated > $O/iso.log 2>$O/iso.err || { tail -20 $O/iso.err; exit 1; }
python -c "import json;d=json.load(open('$O/iso.log'));print('isolated',d['isolated'])"
echo ALLOK
