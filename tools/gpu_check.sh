#!/bin/bash
# One GPU round: parity tests, bench, rocprofv3 kernel-trace stats.  Stops at the first crash/timeout.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o bench --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-north-star > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
rc=$?
echo "rocprof rc=$rc"
exit $rc
