#!/bin/bash
# C2 gram ablations (time-major, 100k x 200): default / no per-step compute / 2 time segments / no contraction
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02z}
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
mkdir -p $O
for v in default ${VARIANTS:-GNOCOMP GNS2 GNOGPH}; do
  if [ $v = default ]; then unset INSITE_LIB_OVERRIDE; else export INSITE_LIB_OVERRIDE=$A/libinsite_hip_$v.so; fi
  for op in gram sindy_fit; do
    timeout -k 10 120 python tools/kbench.py --op $op --layout time --iters 50 > $O/${v}_$op.json 2>$O/${v}_$op.err || { tail -5 $O/${v}_$op.err; exit 1; }
    echo "$v $op $(cat $O/${v}_$op.json | tr -d '\n' | cut -c1-200)"
  done
done
echo ALLOK
