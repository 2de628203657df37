set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04_coop_pmc
mkdir -p $O
timeout -k 10 120 python3 $R/tools/coop_prof.py > $O/plain.log 2>&1 && cat $O/plain.log &&
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -d $O/p1 -o run --output-format csv -- python3 $R/tools/coop_prof.py > $O/p1.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC -d $O/p2 -o run --output-format csv -- python3 $R/tools/coop_prof.py > $O/p2.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INST_CYCLES_SALU SQ_IFETCH SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_FLAT -d $O/p3 -o run --output-format csv -- python3 $R/tools/coop_prof.py > $O/p3.log 2>&1 &&
cd $R && python3 tools/pmc_summary.py $O | grep -A2 coop
