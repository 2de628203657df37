set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
for L in time time_bits; do
  timeout -k 10 120 python tools/kbench.py --op rollout --layout $L --iters 20 >> gpurun_out/kb.log
  timeout -k 10 120 python tools/kbench.py --op rollout --layout $L --patients 1000000 --T 500 --iters 10 >> gpurun_out/kb.log
done
cat gpurun_out/kb.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
tail -1 gpurun_out/bench.log
