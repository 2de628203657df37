#!/bin/bash
# Two-rank rehearsal on a one-GPU box (gloo, both ranks on cuda:0): torchrun-launched C2 pipeline, the
# self-spawning `bench.py --gpus 2` path, and sharded C5
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${OUT:-r02ae}
mkdir -p $O
export INSITE_REHEARSE_ONE_GPU=1 INSITE_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29555 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline > $O/torchrun_c2.log 2>&1 || { tail -30 $O/torchrun_c2.log; exit 1; }
grep '^{' $O/torchrun_c2.log | cut -c1-300
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline > $O/self_c2.log 2>&1 || { tail -30 $O/self_c2.log; exit 1; }
grep '^{' $O/self_c2.log | cut -c1-300
timeout -k 10 300 python bench.py --gpus 2 --config c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/self_c5.log 2>&1 || { tail -30 $O/self_c5.log; exit 1; }
grep '^{' $O/self_c5.log | cut -c1-300
echo ALLOK
