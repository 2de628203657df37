#!/bin/bash
# GPU recipe (round 6): the new GPU tests (RK45 binned by attempts, the claimed gram tail's determinism), then the C5
# line binned by n_obs vs by the previous step's attempt counts, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_f${TAG}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rk45.py tests/test_gpu_deferred.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
show() { python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline',{}); k=d.get('rk45',{}); p=d.get('parity') or {}
print(sys.argv[2], round(d['ms_per_step'],5), round(r.get('avg_launch_ms',0),5), round(r.get('frac',0),4), round(k.get('attempts_max_over_mean_per_wave',0),4), p.get('attempts_equal_frac'), p.get('y_rmse'))" $1 $2; }
for rep in 1 2; do
  for b in nobs attempts; do
    extra="--no-parity"; [ $rep = 2 ] && [ $b = attempts ] && extra=""
    timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --rk45-bin $b $extra > $O/c5_${b}_$rep.jsonl 2> $O/c5_${b}_$rep.err || { echo "c5 $b failed"; tail -5 $O/c5_${b}_$rep.err; exit 1; }
    show $O/c5_${b}_$rep.jsonl c5_$b
  done
done
echo FDONE
