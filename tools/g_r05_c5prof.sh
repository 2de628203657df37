# GPU recipe (round 5): rocprofv3 kernel trace + stats of the C5 line (the binning kernels beside the RK45 kernel)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r05_c5prof
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --no-cpu-baseline --no-parity --steps 10 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
f=$(ls $O/trace/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find $O/trace -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:12]: print(r.get('Name','')[:70], r.get('Calls'), r.get('AverageNs'), r.get('Percentage'))" $f
