#!/bin/bash
# f64 MFMA shape throughput probe + C3 baseline (bench + kernel stats)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02l}
mkdir -p $O
timeout -k 10 60 ./tools/probe/mfma_rate > $O/mfma_rate.txt 2>&1 || { cat $O/mfma_rate.txt; exit 1; }
cat $O/mfma_rate.txt
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline > $O/c3.log 2>$O/c3.err || { tail -20 $O/c3.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --config c3 --no-cpu-baseline --steps 3 --warmup 1 > $O/c3_prof.log 2>&1 || { tail -20 $O/c3_prof.log; exit 1; }
echo ALLOK
