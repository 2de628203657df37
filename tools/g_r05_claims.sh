# GPU recipe (round 5): the deferred C2 step with the per-XCD-slot claimed rollout tail (variant builds from
# tools/build_variant.sh, INSITE_DEF_RSTATIC / INSITE_DEF_RCHUNK) against the static split, interleaved; then the
# deferred / fused parity tests on one claimed build.  usage: VARS="r800c2 ..." bash tools/g_r05_claims.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_claims${TAG}
mkdir -p $O
AB=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
for rep in 1 2; do
  for v in default ${VARS}; do
    if [ "$v" = default ]; then L=""; else L="$AB/libinsite_hip_$v.so"; fi
    INSITE_LIB_OVERRIDE=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --no-north-star --steps ${STEPS:-100} > $O/bench_${v}_$rep.jsonl 2> $O/bench_${v}_$rep.err || { echo "bench $v failed"; tail -5 $O/bench_${v}_$rep.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],5), 'frac', round(d['roofline']['frac'],4))" $O/bench_${v}_$rep.jsonl $v
  done
done
if [ -n "$TESTV" ]; then
  INSITE_LIB_OVERRIDE=$AB/libinsite_hip_$TESTV.so timeout -k 10 600 python -u -m pytest tests/test_gpu_deferred.py tests/test_gpu_fused.py tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_$TESTV.txt 2>&1 || { tail -30 $O/tests_$TESTV.txt; exit 1; }
  tail -2 $O/tests_$TESTV.txt
fi
