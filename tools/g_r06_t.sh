#!/bin/bash
# GPU recipe (round 6): PMC traffic (FETCH_SIZE / WRITE_SIZE passes) of the C2 step, the north-star step and the INSITE
# M = 3 row kernel on the final tree, then the north-star timing variance probe (tools/ns_variance.py: two allocations x
# two timings per process, three processes, the last with a 24-GB caching-allocator reservation first).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_traffic${TAG}
mkdir -p $O
if [ -z "$SKIP_PMC" ]; then
CONFIGS="${TCONF:-c2:--no-north-star --no-c3-block;ns:--config ns;insite:--config insite --insite-only-binned}" OUT=r06_traffic${TAG}/t PMC_LIMIT=240 bash tools/g_traffic.sh || exit 1
fi
for i in 1 2; do
  timeout -k 10 300 python tools/ns_variance.py > $O/nsvar_$i.json 2> $O/nsvar_$i.err || { tail -5 $O/nsvar_$i.err; exit 1; }
  cat $O/nsvar_$i.json
done
timeout -k 10 300 python tools/ns_variance.py --prealloc > $O/nsvar_pre.json 2> $O/nsvar_pre.err || { tail -5 $O/nsvar_pre.err; exit 1; }
cat $O/nsvar_pre.json
echo TDONE
