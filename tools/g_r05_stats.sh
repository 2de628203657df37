# GPU recipe (round 5, final tree): rocprofv3 kernel stats of the secondary lines whose kernels changed this round
# (C5, INSITE, INSITE 4-arm, C3), each beside its bench line's own event timing.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r05_stats
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in ${LINES:-c5 insite insite4 c3}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/$c -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --no-cpu-baseline --no-parity > $O/$c.jsonl 2> $O/$c.log || { echo "prof $c failed"; tail -5 $O/$c.log; exit 1; }
  echo "prof $c ok"
done
