set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
for L in patient time; do
  for OP in gram sindy_fit rollout; do
    timeout -k 10 120 python tools/kbench.py --op $OP --layout $L --iters 50 >> gpurun_out/kb.log
  done
  timeout -k 10 120 python tools/kbench.py --op gram --layout $L --patients 1000000 --T 500 --iters 10 >> gpurun_out/kb.log
done
cat gpurun_out/kb.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1
cat gpurun_out/bench.log | tail -1
