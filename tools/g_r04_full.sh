set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_full
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04_full/test_gpu_all.txt 2>&1 || { tail -40 gpurun_out/r04_full/test_gpu_all.txt; exit 1; }
tail -3 gpurun_out/r04_full/test_gpu_all.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_full/smoke.txt 2>&1 || { tail -20 gpurun_out/r04_full/smoke.txt; exit 1; }
tail -3 gpurun_out/r04_full/smoke.txt
timeout -k 10 300 python bench.py > gpurun_out/r04_full/bench_default.jsonl 2> gpurun_out/r04_full/bench_default.err || { tail -20 gpurun_out/r04_full/bench_default.err; exit 1; }
cat gpurun_out/r04_full/bench_default.jsonl
# C2 deferred: gram / rollout block split sweep (cold rotating cohorts, the default N = 1 schedule)
for G in 192 224 240 272 288 320; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --gram-blocks $G --steps 40 --warmup 5 > gpurun_out/r04_full/c2_gb$G.jsonl 2>/dev/null || exit 1
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('gram_blocks', sys.argv[2], round(d['ms_per_step'],5), round(d['roofline']['frac'],4))" gpurun_out/r04_full/c2_gb$G.jsonl $G
done
timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --steps 40 --warmup 5 > gpurun_out/r04_full/c2_default.jsonl 2>/dev/null && python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('gram_blocks default', d['config'].get('gram_blocks'), round(d['ms_per_step'],5), round(d['roofline']['frac'],4))" gpurun_out/r04_full/c2_default.jsonl
