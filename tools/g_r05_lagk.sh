# GPU recipe (round 5): lagged step bucket size (--pipe-k) x all-reduce delay, single-rank RCCL in the timed region.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_lagk${TAG}
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --no-north-star --steps 96 > $O/deferred_$rep.jsonl 2>$O/deferred_$rep.err || { tail -5 $O/deferred_$rep.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],5), round(d['roofline']['avg_launch_ms'],5))" $O/deferred_$rep.jsonl deferred
  for k in 4 8 16; do for d in 0 1; do
    timeout -k 10 200 python bench.py --mode lagged --force-collective --pipe-k $k --lag-delay $d --no-cpu-baseline --no-parity --no-north-star --steps 96 > $O/k${k}d${d}_$rep.jsonl 2>$O/k${k}d${d}_$rep.err || { tail -5 $O/k${k}d${d}_$rep.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],5), round(d['roofline']['avg_launch_ms'],5))" $O/k${k}d${d}_$rep.jsonl k${k}d${d}
  done; done
done
