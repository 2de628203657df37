set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_rehearse
mkdir -p $O
for n in 2 4; do
  INSITE_REHEARSE_ONE_GPU=1 INSITE_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2953$n bench.py --gpus $n --steps 10 --warmup 3 > $O/bench_n$n.jsonl 2> $O/bench_n$n.err || { echo "n=$n failed"; tail -20 $O/bench_n$n.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('n', d['n_gpus'], 'ms', round(d['ms_per_step'],4), 'value', '%.3e'%d['value'], d['config'].get('mode'), d['config'].get('parallelism'), {k:v for k,v in (d.get('parity') or {}).items() if k in ('support_equal','coef_linf','y_rmse')})" $O/bench_n$n.jsonl
done
