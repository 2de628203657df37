#!/bin/bash
# C2 bench (batched-event pipeline) + kernel trace/stats
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02r}
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2.log 2>$O/c2.err || { tail -20 $O/c2.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-north-star --mode seq > $O/c2_seq.log 2>$O/c2_seq.err || { tail -20 $O/c2_seq.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-north-star --mode graph > $O/c2_graph.log 2>$O/c2_graph.err || { tail -20 $O/c2_graph.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-north-star > $O/c2_prof.log 2>&1 || { tail -20 $O/c2_prof.log; exit 1; }
echo ALLOK
