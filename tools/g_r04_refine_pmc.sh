set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -d $R/gpurun_out/r04_refine_pmc -o run --output-format csv -- python3 $R/bench.py --config insite --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/r04_refine_pmc.log 2>&1
