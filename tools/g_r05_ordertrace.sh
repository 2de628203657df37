# GPU recipe (round 5): kernel timestamps of the C5 plan loop (order + rollout) on the default and two-pass builds,
# to split the step into kernel time and inter-kernel gaps.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_ordertrace
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/fused -o run -- python3 tools/probe/c5_gap.py > $O/fused.log 2>&1 || { tail -5 $O/fused.log; exit 1; }
INSITE_LIB_OVERRIDE=$A/libinsite_hip_twopass.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/twopass -o run -- python3 tools/probe/c5_gap.py > $O/twopass.log 2>&1 || { tail -5 $O/twopass.log; exit 1; }
find $O -name "*kernel_trace.csv" | head
