set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/t_all.log 2>&1
for L in patient time; do
  timeout -k 10 120 python tools/kbench.py --op rollout --layout $L --iters 50 >> gpurun_out/kb.log
  timeout -k 10 120 python tools/kbench.py --op rollout --layout $L --patients 1000000 --T 500 --iters 10 >> gpurun_out/kb.log
done
timeout -k 10 120 python tools/kbench.py --op gram --iters 50 >> gpurun_out/kb.log
cat gpurun_out/kb.log
tail -3 gpurun_out/t_all.log
