#!/bin/bash
# C5 PMC passes (SQ issue/wait split; HBM fetch; HBM write) + kernel stats on the current build
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02j}
mkdir -p $O
B="python3 bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- $B > $O/c5_prof.log 2>&1 || { tail -20 $O/c5_prof.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $O/pmc_sq -o pmc --output-format csv -- $B > $O/pmc_sq.log 2>&1 || { tail -20 $O/pmc_sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o pmc --output-format csv -- $B > $O/pmc_fetch.log 2>&1 || { tail -20 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o pmc --output-format csv -- $B > $O/pmc_write.log 2>&1 || { tail -20 $O/pmc_write.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d $O/pmc_sq2 -o pmc --output-format csv -- $B > $O/pmc_sq2.log 2>&1 || { tail -20 $O/pmc_sq2.log; exit 1; }
echo ALLOK
