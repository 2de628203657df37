set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_dyn2
timeout -k 10 300 python -u -m pytest tests/test_gpu_insite.py -x -q -k "dynamic or rows_layout" > gpurun_out/r04_dyn2/tests.txt 2>&1 || { tail -30 gpurun_out/r04_dyn2/tests.txt; exit 1; }
tail -2 gpurun_out/r04_dyn2/tests.txt
run() {
  f=gpurun_out/r04_dyn2/$(echo "$@" | tr ' =' '__').jsonl
  timeout -k 10 200 env "$@" python bench.py --config insite --no-cpu-baseline --steps 5 --warmup 2 > $f 2>/dev/null &&
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],3), round(d['roofline']['avg_launch_ms'],3))" $f "$*"
}
run INSITE_REFINE_DYN=0 &&
run INSITE_REFINE_DYN=1 &&
run INSITE_REFINE_DYN_REFILL=4 &&
run INSITE_REFINE_DYN_REFILL=16 &&
run INSITE_REFINE_DYN_BLOCKS=512 &&
run INSITE_REFINE_DYN_BLOCKS=1536 &&
run INSITE_REFINE_DYN_REFILL=2 &&
run INSITE_REFINE_DYN_REFILL=32
