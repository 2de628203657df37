#!/bin/bash
# C3 gram_ms PMC passes: issue/wait split + MFMA busy; instruction mix + LDS conflicts + clock
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02m}
mkdir -p $O
B="python3 bench.py --config c3 --no-cpu-baseline --steps 1 --warmup 1"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 -d $O/pmc1 -o pmc --output-format csv -- $B > $O/pmc1.log 2>&1 || { tail -20 $O/pmc1.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAVES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT -d $O/pmc2 -o pmc --output-format csv -- $B > $O/pmc2.log 2>&1 || { tail -20 $O/pmc2.log; exit 1; }
echo ALLOK
