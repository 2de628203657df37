#!/bin/bash
# Two-rank rehearsal of bench.py's multi-GPU step on a one-GPU box (gloo, both ranks on cuda:0).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export INSITE_REHEARSE_ONE_GPU=1 INSITE_DIST_BACKEND=gloo
for m in pipeline seq; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29555 bench.py --gpus 2 --steps 10 --warmup 3 --mode $m --no-cpu-baseline > gpurun_out/rehearse2_$m.log 2>&1 || { tail -30 gpurun_out/rehearse2_$m.log; exit 1; }
  grep '^{' gpurun_out/rehearse2_$m.log | cut -c1-400
done
