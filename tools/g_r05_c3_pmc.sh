# GPU recipe (round 5): C3 gram_ms4_kernel SQ issue / wait / LDS / MFMA counters (one rocprofv3 --pmc pass per
# counter group), optionally on a variant library (LIBV); the counter list of the box first (rocprofv3 -L).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_c3_pmc${TAG}
mkdir -p $O
if [ -n "$LIBV" ]; then export INSITE_LIB_OVERRIDE=$R/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate/libinsite_hip_$LIBV.so; fi
B="$R/bench.py --config c3 --no-cpu-baseline --no-parity --steps 3 --warmup 1"
if [ -n "$LIST" ]; then timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true; fi
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES -d $O/p1 -o run --output-format csv -- python3 $B > $O/p1.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_MISC -d $O/p2 -o run --output-format csv -- python3 $B > $O/p2.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MFMA SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_LDS SQ_INSTS_BRANCH -d $O/p3 -o run --output-format csv -- python3 $B > $O/p3.log 2>&1 &&
python3 $R/tools/pmc_summary.py $O > $O/summary.json && python3 -c "
import json,sys
d=json.load(open('$O/summary.json'))
for run,v in d.items():
  for k,x in v.items():
    if 'gram_ms4' in k: print(run, k.split()[-1], round(x['mean']))"
