#!/bin/bash
# C5 after gating the bit-exact min_step on a wave ballot: RK45 parity (attempt counts vs the oracle) + C5 line x2
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02at}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rk45.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/c5_$r.log 2>$O/err || { tail -5 $O/err; exit 1; }
  python -c "import json;d=json.loads(open('$O/c5_$r.log').read().splitlines()[-1]);print('c5 ms',round(d['ms_per_step'],4),'roll',round(d['roofline']['avg_launch_ms'],4),d['rk45']['mean_attempts_per_patient'])"
done
echo ALLOK
