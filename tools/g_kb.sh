#!/bin/bash
# Standalone kernel timings at C2 (and the 1M x 500 rollout) + the non-pipelined bench.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/kb.log
for a in "--op rollout --layout time_bits" "--op rollout --layout time" "--op gram --layout time" "--op sindy_fit --layout time" \
         "--op rollout --layout time_bits --patients 1000000 --T 500" ${KB_EXTRA:-}; do
  timeout -k 10 120 python tools/kbench.py $a --iters 50 >> gpurun_out/kb.log
done
cat gpurun_out/kb.log
timeout -k 10 300 python bench.py --mode seq --no-cpu-baseline --no-north-star > gpurun_out/bench_np.log 2>&1
tail -1 gpurun_out/bench_np.log
