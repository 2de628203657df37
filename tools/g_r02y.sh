#!/bin/bash
# INSITE refinement with rows binned by seq_len: parity tests + bench (binned vs identity order)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02y}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_insite.py tests/test_gpu_reference.py tests/test_gpu_plugin.py tests/test_gpu_fused.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --config insite > $O/insite.log 2>$O/insite.err || { tail -20 $O/insite.err; exit 1; }
python -c "import json;d=json.loads(open('$O/insite.log').read().splitlines()[-1]);print('insite ms',round(d['ms_per_step'],3),'identity',round(d['insite']['identity_order_ms_per_step'],3), d['insite']['mean_bfgs_iterations'], d.get('cpu_baseline',{}).get('value'))"
echo ALLOK
