# GPU recipe (round 5): SQ issue / wait / LDS / memory-instruction counters and FETCH / WRITE of the INSITE line's
# kernels (two-to-four rocprofv3 --pmc passes, one counter group each), optionally on a variant library (LIBV).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_refine_pmc${TAG}
mkdir -p $O
if [ -n "$LIBV" ]; then export INSITE_LIB_OVERRIDE=$R/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate/libinsite_hip_$LIBV.so; fi
B="$R/bench.py --config ${CFG:-insite} --no-cpu-baseline --no-parity --steps 3 --warmup 1 ${BARGS:---insite-only-binned}"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -d $O/p1 -o run --output-format csv -- python3 $B > $O/p1.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_MISC -d $O/p2 -o run --output-format csv -- python3 $B > $O/p2.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/p3 -o run --output-format csv -- python3 $B > $O/p3.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/p4 -o run --output-format csv -- python3 $B > $O/p4.log 2>&1 &&
python3 $R/tools/pmc_summary.py $O ${KPAT:-insite_refine_kernel} > $O/summary.json && cat $O/summary.json
