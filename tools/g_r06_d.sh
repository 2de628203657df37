#!/bin/bash
# GPU recipe (round 6): the adaptive claimed gram tail (INSITE_DEF_DYN=2: claimed at the north-star shape, static at
# C2's) -- the deferred / fused / dist GPU tests on this tree, then the north-star line A/B, interleaved: this tree vs
# never-claimed (nodyn) vs the claimed tail's share (t100 / t250 / t350 per mille; this tree: 150).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_d${TAG}
mkdir -p $O
AB=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
show() { python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline',{}); p=d.get('parity') or {}
print(sys.argv[2], round(d['ms_per_step'],5), round(r.get('avg_launch_ms',0),5), round(r.get('frac',0),4), p.get('support_equal'), p.get('coef_linf'))" $1 $2; }
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_deferred.py tests/test_gpu_fused.py tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_def.txt 2>&1 || { tail -30 $O/tests_def.txt; exit 1; }
tail -2 $O/tests_def.txt
fi
timeout -k 10 300 python bench.py --config ns > $O/ns_parity.jsonl 2> $O/ns_parity.err || { tail -5 $O/ns_parity.err; exit 1; }
show $O/ns_parity.jsonl ns_default_with_parity
for rep in 1 2 3; do
  for v in default ${NSVARS:-nodyn t100 t250 t350}; do
    if [ "$v" = default ]; then L=""; else L="$AB/libinsite_hip_$v.so"; fi
    INSITE_LIB_OVERRIDE=$L timeout -k 10 300 python bench.py --config ns --no-parity --ns-steps 20 > $O/ns_${v}_$rep.jsonl 2> $O/ns_${v}_$rep.err || { echo "ns $v failed"; tail -5 $O/ns_${v}_$rep.err; exit 1; }
    show $O/ns_${v}_$rep.jsonl ns_$v
  done
done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --no-north-star --no-c3-block --steps 100 > $O/c2_default.jsonl 2> $O/c2_default.err || { tail -5 $O/c2_default.err; exit 1; }
show $O/c2_default.jsonl c2_default
echo DDONE
