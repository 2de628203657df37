set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_full
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04_full/test_gpu_all.txt 2>&1 || { tail -40 gpurun_out/r04_full/test_gpu_all.txt; exit 1; }
tail -3 gpurun_out/r04_full/test_gpu_all.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_full/smoke.txt 2>&1 || { tail -20 gpurun_out/r04_full/smoke.txt; exit 1; }
tail -3 gpurun_out/r04_full/smoke.txt
timeout -k 10 300 python bench.py > gpurun_out/r04_full/bench_default.jsonl 2> gpurun_out/r04_full/bench_default.err || { tail -20 gpurun_out/r04_full/bench_default.err; exit 1; }
cat gpurun_out/r04_full/bench_default.jsonl
