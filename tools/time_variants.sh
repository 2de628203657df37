#!/bin/bash
# Time one op across the tuning/ablation builds (interleaved rounds in separate processes).
cd "$GRAFT_REPO_ROOT" || exit 1
OP=${OP:-gram}
# every EXTRA_SETS entry (";"-separated) is timed as its own configuration
IFS=';' read -ra SETS <<< "${EXTRA_SETS:-${EXTRA:-}}"
for EXTRA in "${SETS[@]}"; do
for round in 1 2; do
  timeout -k 10 120 python tools/kbench.py --op $OP --iters ${ITERS:-50} ${EXTRA:-} || exit $?
  for v in ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate/*.so; do
    INSITE_LIB_OVERRIDE="$PWD/$v" timeout -k 10 120 python tools/kbench.py --op $OP --iters ${ITERS:-50} ${EXTRA:-} || exit $?
  done
done
done
