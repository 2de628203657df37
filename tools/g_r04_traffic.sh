set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CONFIGS="c2:--no-north-star;c4:--config c4 --T 60;c5:--config c5;c3:--config c3;f4:--config f4;insite:--config insite;insite4:--config insite4" OUT=r04_traffic PMC_LIMIT=240 bash tools/g_traffic.sh || exit 1
# C5: instruction breakdown of the rollout kernel (one SQ pass, 8 counters)
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -d gpurun_out/r04_c5_sq -o run --output-format csv -- python3 bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r04_c5_sq.log 2>&1 && echo C5SQ ok
