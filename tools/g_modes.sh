#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for m in graph seq pipeline; do
  timeout -k 10 300 python bench.py --mode $m --no-cpu-baseline --no-north-star --steps 50 > gpurun_out/bench_$m.log 2>&1 || { tail -20 gpurun_out/bench_$m.log; exit 1; }
  tail -1 gpurun_out/bench_$m.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', d['ms_per_step'], d['value'], d['roofline']['avg_launch_ms'], d['discovery']['avg_ms'])"
done
