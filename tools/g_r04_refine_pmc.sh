set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -d $R/gpurun_out/r04_refine_pmc_v3 -o run --output-format csv -- python3 $R/bench.py --config insite --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/r04_refine_pmc_v3.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC -d $R/gpurun_out/r04_refine_pmc_v32 -o run --output-format csv -- python3 $R/bench.py --config insite --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/r04_refine_pmc_v32.log 2>&1 &&
echo done
