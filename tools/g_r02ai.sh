#!/bin/bash
# one-pass C4 fits (insite_gram_moments_f64 + insite_fit_per_patient_moments_f64): tests, C4 lines
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02ai}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_moments.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() { n=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/$n.log 2>$O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/$n.log').read().splitlines()[-1]);print('$n ms',round(d['ms_per_step'],4),'disc',d['discovery'],'pp',d['per_patient_fit']['avg_ms'],'roll',d['roofline']['avg_launch_ms'],d['config']['global_support'])"; }
run c4_T60 --config c4
run c4_T500 --config c4 --T 500 --no-cpu-baseline
echo ALLOK
