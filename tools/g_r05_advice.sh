# GPU recipe (round 5): the ADVICE follow-ups' GPU tests (slot fingerprint, dynamic-assignment knobs), then the
# cooperative kernel's SQ / traffic counters on the insite4 line.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_advice
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_deferred.py tests/test_gpu_insite.py -m gpu -x -q --timeout 300 --timeout-method thread -k "deferred or dynamic" > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
CFG=insite4 BARGS=" " KPAT=insite_refine_coop_kernel TAG=_coop2 bash tools/g_r05_refine_pmc.sh > $O/coop_pmc.txt 2>&1 || { tail -5 $O/coop_pmc.txt; exit 1; }
echo PMCOK
# C5: FETCH_SIZE / WRITE_SIZE calibration on its access shape (window refills, 64-B output sectors), then the
# RK45 kernel's own counters on the C5 line
cd /tmp && export TMPDIR=/tmp
P=$GRAFT_REPO_ROOT/gpurun_out/r05_c5cal
mkdir -p $P
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $C -d $P/probe_$C -o run --output-format csv -- $GRAFT_REPO_ROOT/tools/probe/bin/window_probe 1000000 > $P/probe_$C.log 2>&1 || { tail -5 $P/probe_$C.log; exit 1; }
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $P > $P/probe_summary.json && cat $P/probe_*.log | grep rows | head -1
cd $GRAFT_REPO_ROOT && CFG=c5 BARGS=" " KPAT=rollout_rk45 TAG=_c5 bash tools/g_r05_refine_pmc.sh > $O/c5_pmc.txt 2>&1 || { tail -5 $O/c5_pmc.txt; exit 1; }
echo C5OK
