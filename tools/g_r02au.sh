#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate --pmc passes) of the fused step kernel on the C2 cohort
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02au}
mkdir -p $O
timeout -k 10 120 python3 tools/kbench.py --op fused --layout time_bits --iters 20 > $O/kb.json 2>$O/kb.err || { tail -5 $O/kb.err; exit 1; }
cat $O/kb.json
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d "$GRAFT_REPO_ROOT/$O/fused_$C" -o run --output-format csv -- python3 tools/kbench.py --op fused --layout time_bits --iters 10 > $O/fused_$C.log 2>&1 || exit 1
done
python3 tools/pmc_summary.py $O > $O/summary.json && cat $O/summary.json && echo ALLOK
