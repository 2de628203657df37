#!/bin/bash
# bench.py (ARGS) once per library build -- the default and every lib/ablate variant -- ROUNDS times, interleaved;
# one "<lib> <ms_per_step> <roofline frac>" line each.  Tuning evidence only.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${OUT:-variants}
mkdir -p $O
L=ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in default $L/ablate/*.so; do
    name=$(basename $v .so)
    if [ "$v" = default ]; then ov=""; else ov="$PWD/$v"; fi
    INSITE_LIB_OVERRIDE=$ov timeout -k 10 200 python bench.py ${ARGS:---no-cpu-baseline --no-north-star} > $O/b_${name}_$r.json 2>$O/b_${name}_$r.err || { echo "bench failed: $name"; tail -5 $O/b_${name}_$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],5), round(d['roofline']['frac'],4))" $O/b_${name}_$r.json $name | tee -a $O/summary.txt
  done
done
echo VARIANTSOK
