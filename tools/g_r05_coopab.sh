set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_coop${TAG:-_pipe}
mkdir -p $O
TAG=${TAG:-_pipe} bash tools/g_r05_coop.sh || exit 1
INSITE_LIB_OVERRIDE=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate/libinsite_hip_${VAR:-nopipe}.so timeout -k 10 500 python bench.py --config insite4 --no-cpu-baseline --no-parity > $O/bench_${VAR:-nopipe}.jsonl 2> $O/bench_${VAR:-nopipe}.err || { tail -5 $O/bench_${VAR:-nopipe}.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k,v in d['models'].items(): print(sys.argv[1], k, round(v['ms_per_step'],3), 'kern', round(v['kernel_ms'],3))" $O/bench_${VAR:-nopipe}.jsonl
