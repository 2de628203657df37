#!/bin/bash
# Phase timestamps (INSITE_TIMING build in lib/ablate) of the gram and the fused step with cold caches.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${OUT:-timing}
mkdir -p $O
L="$PWD/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate/libinsite_hip_TIMING.so"
for op in ${OPS:-gram fused}; do
  INSITE_LIB_OVERRIDE="$L" timeout -k 10 120 python tools/kbench.py --op $op --layout time_bits --cold --timing --iters 10 ${EXTRA:-} >> $O/timing.jsonl || exit 1
done
echo TIMINGOK
