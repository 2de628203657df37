#!/bin/bash
# GPU recipe (round 6): (1) the claimed gram tail (INSITE_DEF_DYN variant builds, tools/build_variant.sh) against the
# oracle; (2) C2 step A/B: the round-5 insite_hip.hip, this tree's default, the DYN variants, interleaved; (3) the
# north-star line (--config ns) unprofiled; (4) the lagged step's split: deferred | lagged without
# the collective | lagged + single-rank RCCL in order | lagged + RCCL async, K = 16.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_b${TAG}
mkdir -p $O
AB=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
show() { python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline',{}); print(sys.argv[2], round(d['ms_per_step'],5), round(r.get('avg_launch_ms',0),5), round(r.get('frac',0),4))" $1 $2; }
if [ -n "$TESTV" ]; then
  INSITE_LIB_OVERRIDE=$AB/libinsite_hip_$TESTV.so timeout -k 10 600 python -u -m pytest tests/test_gpu_deferred.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_$TESTV.txt 2>&1 || { tail -30 $O/tests_$TESTV.txt; exit 1; }
  tail -2 $O/tests_$TESTV.txt
fi
for rep in 1 2; do
  for v in default ${VARS}; do
    if [ "$v" = default ]; then L=""; else L="$AB/libinsite_hip_$v.so"; fi
    INSITE_LIB_OVERRIDE=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --no-north-star --no-c3-block --steps ${STEPS:-100} > $O/c2_${v}_$rep.jsonl 2> $O/c2_${v}_$rep.err || { echo "bench $v failed"; tail -5 $O/c2_${v}_$rep.err; exit 1; }
    show $O/c2_${v}_$rep.jsonl c2_$v
  done
done
if [ -n "$NSV" ]; then
  for v in default $NSV; do
    if [ "$v" = default ]; then L=""; else L="$AB/libinsite_hip_$v.so"; fi
    INSITE_LIB_OVERRIDE=$L timeout -k 10 300 python bench.py --config ns --no-parity > $O/ns_${v}.jsonl 2> $O/ns_${v}.err || { echo "ns $v failed"; tail -5 $O/ns_${v}.err; exit 1; }
    show $O/ns_${v}.jsonl ns_$v
  done
fi
if [ -n "$LAG" ]; then
  for rep in 1 2; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --no-north-star --no-c3-block --steps 96 > $O/lag_deferred_$rep.jsonl 2>$O/lag_deferred_$rep.err || { tail -5 $O/lag_deferred_$rep.err; exit 1; }
    show $O/lag_deferred_$rep.jsonl deferred
    timeout -k 10 200 python bench.py --mode lagged --no-cpu-baseline --no-parity --no-north-star --no-c3-block --steps 96 > $O/lag_nocoll_$rep.jsonl 2>$O/lag_nocoll_$rep.err || { tail -5 $O/lag_nocoll_$rep.err; exit 1; }
    show $O/lag_nocoll_$rep.jsonl lagged_no_collective
    timeout -k 10 200 python bench.py --mode lagged --force-collective --lag-k 16 --lag-delay 0 --no-cpu-baseline --no-parity --no-north-star --no-c3-block --steps 96 > $O/lag_inorder_$rep.jsonl 2>$O/lag_inorder_$rep.err || { tail -5 $O/lag_inorder_$rep.err; exit 1; }
    show $O/lag_inorder_$rep.jsonl lagged_rccl_inorder
    timeout -k 10 200 python bench.py --mode lagged --force-collective --lag-k 16 --lag-delay 1 --no-cpu-baseline --no-parity --no-north-star --no-c3-block --steps 96 > $O/lag_async_$rep.jsonl 2>$O/lag_async_$rep.err || { tail -5 $O/lag_async_$rep.err; exit 1; }
    show $O/lag_async_$rep.jsonl lagged_rccl_async
  done
fi
echo ALLDONE
