#!/bin/bash
# C2 fused-step split sweep with rotated cohorts (+ isolated halves), achievable-bandwidth probe, the
# default line's rocprofv3 kernel summary and the C5 WRITE_SIZE pass.  Each GPU step has its own limit.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-c2sweep}
mkdir -p $O
timeout -k 10 120 python tools/bwprobe.py > $O/bwprobe.json 2>$O/bwprobe.err || { tail $O/bwprobe.err; exit 1; }
cat $O/bwprobe.json
timeout -k 10 200 python bench.py --no-cpu-baseline --no-north-star --isolated > $O/iso.log 2>$O/iso.err || { tail $O/iso.err; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/iso.log').read().strip().splitlines()[-1]); print('iso', d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('isolated'))"
for G in ${GBS:-256 288 336 368 400}; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-north-star --gram-blocks $G > $O/g$G.log 2>$O/g$G.err || { tail $O/g$G.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/g$G.log').read().strip().splitlines()[-1]); print('G=$G', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/bench_prof.log 2>&1 || { tail -20 $O/bench_prof.log; exit 1; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
[ -n "$T" ] && python tools/rocprof_by_grid.py "$T" $O/bench_kernels_by_grid.csv && head -8 $O/bench_kernels_by_grid.csv
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/c5_write -o run --output-format csv -- python3 bench.py --config c5 --no-cpu-baseline --steps 5 --warmup 2 > $O/c5_write.log 2>&1 || { tail -20 $O/c5_write.log; exit 1; }
echo ALLOK
