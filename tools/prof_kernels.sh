#!/bin/bash
# Kernel-level profiling: timings of ablation builds + PMC counter passes (one pass per group).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
OP=${OP:-gram}
ARGS="--op $OP --iters ${ITERS:-50} ${EXTRA:-}"
timeout -k 10 120 python tools/kbench.py $ARGS > gpurun_out/pmc/kb_default.json 2>/dev/null || exit $?
for v in gpurun_out/../ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate/*.so; do
  [ -e "$v" ] || continue
  n=$(basename "$v" .so)
  INSITE_LIB_OVERRIDE="$PWD/$v" timeout -k 10 120 python tools/kbench.py $ARGS > gpurun_out/pmc/kb_$n.json 2>/dev/null || exit $?
done
cat gpurun_out/pmc/kb_*.json
[ -n "$LIST" ] && { timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true; }
cd /tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE" ${PMC_EXTRA:-}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/p$i" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/kbench.py" --op $OP --iters 10 ${EXTRA:-} > "$GRAFT_REPO_ROOT/gpurun_out/pmc/p$i.log" 2>&1 || exit $?
done
echo done
