#!/bin/bash
# GPU recipe (round 6): INSITE 4-arm line, lanes binned by seq_len vs by seq_len + the previous step's evaluation
# counts (--insite-order), interleaved on one box; the refinement GPU tests first.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_insite4${TAG}
mkdir -p $O
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_insite.py tests/test_gpu_refine_general.py tests/test_gpu_reference_segments.py tests/test_gpu_plugin.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
fi
for rep in $(seq 1 ${REPS:-1}); do
  for o in ${ORDERS:-seq_len nfev}; do
    ENVP=""; oo=$o
    if [ "$o" = nfev_prep ]; then ENVP="INSITE_REFINE_ROWS=0"; oo=nfev; fi
    if [ "$o" = nfev_coop8 ]; then ENVP="INSITE_LIB_OVERRIDE=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate/libinsite_hip_coop8rows.so"; oo=nfev; fi
    env $ENVP timeout -k 10 600 python bench.py --config insite4 --no-cpu-baseline ${EXTRA:-} --insite-order $oo > $O/insite4_${o}_$rep.jsonl 2> $O/insite4_${o}_$rep.err || { echo "insite4 $o failed"; tail -5 $O/insite4_${o}_$rep.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); m=d.get('models') or d.get('insite4') or {}
for k,v in (m.items() if isinstance(m,dict) else []):
    if isinstance(v,dict) and 'ms_per_step' in v: print(sys.argv[2], k, round(v['ms_per_step'],3), 'kern', round(v.get('kernel_ms',0),3), 'div', round(v.get('wave_divergence',{}).get('max_over_mean_evaluations',0),3), 'eq', v.get('equal_to_nfev_route'), (v.get('parity') or {}).get('status_equal_frac'))
print(sys.argv[2], 'line', round(d['ms_per_step'],3))" $O/insite4_${o}_$rep.jsonl $o
  done
done
echo I4DONE
