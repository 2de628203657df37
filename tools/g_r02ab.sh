#!/bin/bash
# gram phase timestamps (INSITE_TIMING build) for the C2 time-major gram, default vs no G-phase
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02ab}
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
mkdir -p $O
INSITE_LIB_OVERRIDE=$A/libinsite_hip_TIMING.so timeout -k 10 120 python tools/kbench.py --op gram --layout time --iters 20 --timing > $O/timing_gram.txt 2>&1 || { tail -5 $O/timing_gram.txt; exit 1; }
cat $O/timing_gram.txt
INSITE_LIB_OVERRIDE=$A/libinsite_hip_TIMING.so timeout -k 10 120 python tools/kbench.py --op rollout --layout time_bits --iters 20 --timing > $O/timing_roll.txt 2>&1 || { tail -5 $O/timing_roll.txt; exit 1; }
cat $O/timing_roll.txt
INSITE_LIB_OVERRIDE=$A/libinsite_hip_GNOGPH.so timeout -k 10 120 python tools/kbench.py --op gram --layout time --iters 20 > $O/nogph.txt 2>&1 || { tail -5 $O/nogph.txt; exit 1; }
cat $O/nogph.txt
echo ALLOK
