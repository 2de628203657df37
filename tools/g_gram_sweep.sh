#!/bin/bash
# Cold-cache A/B of the gram / fused step across the tuning builds in lib/ablate (tools/build_ablation.sh):
# kbench --cold evicts L2 and the Infinity Cache before every timed call.  One JSON line per (lib, op).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${OUT:-sweep}
mkdir -p $O
for op in ${OPS:-gram fused}; do
  for v in default ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate/*.so; do
    if [ "$v" = default ]; then
      timeout -k 10 120 python tools/kbench.py --op $op --layout time_bits --cold --iters ${ITERS:-30} >> $O/sweep.jsonl || exit 1
    else
      INSITE_LIB_OVERRIDE="$PWD/$v" timeout -k 10 120 python tools/kbench.py --op $op --layout time_bits --cold --iters ${ITERS:-30} >> $O/sweep.jsonl || exit 1
    fi
  done
done
echo SWEEPOK
