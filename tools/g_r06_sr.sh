#!/bin/bash
# GPU recipe (round 6): the self-resetting lane-order sort (no memset launch) -- RK45 / refinement tests, then the C5
# and INSITE lines on this tree vs the memset build (sr0), interleaved on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_sr${TAG}
mkdir -p $O
AB=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
timeout -k 10 600 python -u -m pytest tests/test_gpu_rk45.py tests/test_gpu_insite.py tests/test_gpu_config_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for rep in 1 2; do
  for v in default sr0; do
    if [ "$v" = default ]; then L=""; else L="$AB/libinsite_hip_$v.so"; fi
    for c in c5 insite; do
      INSITE_LIB_OVERRIDE=$L timeout -k 10 400 python bench.py --config $c --no-cpu-baseline --no-parity > $O/${c}_${v}_$rep.jsonl 2> $O/${c}_${v}_$rep.err || { echo "$c $v failed"; tail -5 $O/${c}_${v}_$rep.err; exit 1; }
      python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline',{})
print(sys.argv[2], round(d['ms_per_step'],5), round(r.get('avg_launch_ms',0) or 0,5))" $O/${c}_${v}_$rep.jsonl ${c}_$v
    done
  done
done
echo SRDONE
