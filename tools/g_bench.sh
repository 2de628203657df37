set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for f in "" "--mode seq"; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-north-star $f > gpurun_out/bench_x.log 2>&1
  tail -1 gpurun_out/bench_x.log
done
