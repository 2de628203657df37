set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_dyn
run() { timeout -k 10 200 env "$@" python bench.py --config insite --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/r04_dyn/$(echo "$@" | tr ' =' '__').jsonl 2>/dev/null && python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],3), round(d['roofline']['avg_launch_ms'],3))" gpurun_out/r04_dyn/$(echo "$@" | tr ' =' '__').jsonl "$*"; }
run INSITE_REFINE_DYN=0 &&
run INSITE_REFINE_DYN=1 &&
run INSITE_REFINE_DYN_RPB=2048 &&
run INSITE_REFINE_DYN_RPB=8192 &&
run INSITE_REFINE_DYN_RPB=2048 INSITE_REFINE_DYN_REFILL=1 &&
run INSITE_REFINE_DYN_RPB=2048 INSITE_REFINE_DYN_REFILL=32 &&
run INSITE_REFINE_DYN_RPB=256
