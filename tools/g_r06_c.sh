#!/bin/bash
# GPU recipe (round 6): the refinement kernels -- (1) cooperative == single-lane and the INSITE GPU tests on this tree
# (the split scan, INSITE_COOP_SCAN_SPLIT); (2) the 4-arm INSITE line, this tree vs the unsplit scan; (3) the M = 3 row
# kernel at 3 waves / SIMD (default, spills) vs 2 (INSITE_REFINE_WPE4=2, no spills), interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_c${TAG}
mkdir -p $O
AB=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_insite.py tests/test_gpu_refine_general.py tests/test_gpu_reference_segments.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_refine.txt 2>&1 || { tail -30 $O/tests_refine.txt; exit 1; }
tail -2 $O/tests_refine.txt
fi
show4() { python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
m=d.get('models') or {}
print(sys.argv[2], round(d['ms_per_step'],4), {k: round(v.get('ms_per_step',0),4) for k,v in m.items()} if isinstance(m,dict) else '', (d.get('parity') or {}).get('status_equal_frac'))" $1 $2; }
for rep in 1 2; do
  for v in default ${VARS4:-coopnosplit}; do
    if [ "$v" = default ]; then L=""; else L="$AB/libinsite_hip_$v.so"; fi
    INSITE_LIB_OVERRIDE=$L timeout -k 10 400 python bench.py --config insite4 --no-cpu-baseline ${NOPAR4:---no-parity} --steps ${STEPS4:-5} > $O/i4_${v}_$rep.jsonl 2> $O/i4_${v}_$rep.err || { echo "insite4 $v failed"; tail -5 $O/i4_${v}_$rep.err; exit 1; }
    show4 $O/i4_${v}_$rep.jsonl i4_$v
  done
  for v in default ${VARS3:-refwpe2}; do
    if [ "$v" = default ]; then L=""; else L="$AB/libinsite_hip_$v.so"; fi
    INSITE_LIB_OVERRIDE=$L timeout -k 10 400 python bench.py --config insite --insite-only-binned --no-cpu-baseline --no-parity --steps ${STEPS3:-10} > $O/i3_${v}_$rep.jsonl 2> $O/i3_${v}_$rep.err || { echo "insite $v failed"; tail -5 $O/i3_${v}_$rep.err; exit 1; }
    show4 $O/i3_${v}_$rep.jsonl i3_$v
  done
done
echo ALLDONE
