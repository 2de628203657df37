#!/bin/bash
# rocprofv3 kernel stats of the F4 segment Gram (default build and one variant)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/segprof
A=ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/segprof/default" -o run --output-format csv -- python3 tools/kbench.py --op gram_seg --patients 1000000 --T 60 --iters 20 > gpurun_out/segprof/default.log 2>&1 || exit 1
for v in ${SEGV:-SEGKC4}; do
  INSITE_LIB_OVERRIDE=$A/libinsite_hip_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/segprof/$v" -o run --output-format csv -- python3 tools/kbench.py --op gram_seg --patients 1000000 --T 60 --iters 20 > gpurun_out/segprof/$v.log 2>&1 || exit 1
done
for f in $(find gpurun_out/segprof -name "*kernel_stats.csv"); do echo "== $f"; grep -E "gram_seg|discovery_finalize" "$f" | cut -c1-60,200- | head; done
