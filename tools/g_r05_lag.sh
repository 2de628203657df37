# GPU recipe (round 5): the N > 1 lagged step at N = 1 with the single-rank RCCL collective in the timed region --
# the bucket all-reduce in order (delay 0) vs overlapped (delay 1) -- against the deferred step; dist tests first.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_lag${TAG}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_deferred.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --no-north-star --steps 100 > $O/deferred_$rep.jsonl 2>$O/deferred_$rep.err || { tail -5 $O/deferred_$rep.err; exit 1; }
  for d in 0 1; do
    timeout -k 10 200 python bench.py --mode lagged --force-collective --lag-delay $d --no-cpu-baseline --no-parity --no-north-star --steps 100 > $O/lag${d}_$rep.jsonl 2>$O/lag${d}_$rep.err || { tail -5 $O/lag${d}_$rep.err; exit 1; }
  done
  for f in deferred_$rep lag0_$rep lag1_$rep; do python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],5), round(d['roofline']['avg_launch_ms'],5))" $O/$f.jsonl $f; done
done
