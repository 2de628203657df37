# GPU recipe (round 5, final tree): the lagged step (K = 16, delay 1, single-rank RCCL in the timed region) against
# the deferred step, alternating, three runs each on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_lagfinal
mkdir -p $O
show() { python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],5), round(d['roofline']['avg_launch_ms'],5))" $1 $2; }
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --no-north-star --steps 96 > $O/deferred_$rep.jsonl 2>$O/deferred_$rep.err || { tail -5 $O/deferred_$rep.err; exit 1; }
  show $O/deferred_$rep.jsonl deferred
  timeout -k 10 200 python bench.py --mode lagged --force-collective --pipe-k 16 --lag-delay 1 --no-cpu-baseline --no-parity --no-north-star --steps 96 > $O/lagged_$rep.jsonl 2>$O/lagged_$rep.err || { tail -5 $O/lagged_$rep.err; exit 1; }
  show $O/lagged_$rep.jsonl lagged
done
