set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_insite.py tests/test_gpu_dist.py tests/test_gpu_refine_general.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04_rows_tests.txt 2>&1 || { tail -30 gpurun_out/r04_rows_tests.txt; exit 1; }
tail -3 gpurun_out/r04_rows_tests.txt
timeout -k 10 300 python bench.py --config insite --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/r04_rows_bench.jsonl 2> gpurun_out/r04_rows_bench.err || { tail -20 gpurun_out/r04_rows_bench.err; exit 1; }
cat gpurun_out/r04_rows_bench.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04_rows_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config insite --no-cpu-baseline --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r04_rows_prof.log 2>&1 || exit 1
bash $GRAFT_REPO_ROOT/tools/g_r04_refine_pmc.sh
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --config insite4 --steps 3 --warmup 1 > gpurun_out/r04_insite4.jsonl 2> gpurun_out/r04_insite4.err || { tail -20 gpurun_out/r04_insite4.err; exit 1; }
cat gpurun_out/r04_insite4.jsonl
