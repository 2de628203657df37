# GPU recipe (round 5): the lagged step with the STLSQ merged into the reduction block (default) vs its own block
# (lagsep variant), K = 16 delay 1, single-rank RCCL in the timed region, against the deferred step; dist tests first.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_lagm
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_deferred.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
show() { python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],5), round(d['roofline']['avg_launch_ms'],5))" $1 $2; }
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --no-north-star --steps 96 > $O/deferred_$rep.jsonl 2>$O/deferred_$rep.err || { tail -5 $O/deferred_$rep.err; exit 1; }
  show $O/deferred_$rep.jsonl deferred
  timeout -k 10 200 python bench.py --mode lagged --force-collective --pipe-k 16 --lag-delay 1 --no-cpu-baseline --no-parity --no-north-star --steps 96 > $O/merged_$rep.jsonl 2>$O/merged_$rep.err || { tail -5 $O/merged_$rep.err; exit 1; }
  show $O/merged_$rep.jsonl merged
  INSITE_LIB_OVERRIDE=$A/libinsite_hip_lagsep.so timeout -k 10 200 python bench.py --mode lagged --force-collective --pipe-k 16 --lag-delay 1 --no-cpu-baseline --no-parity --no-north-star --steps 96 > $O/sep_$rep.jsonl 2>$O/sep_$rep.err || { tail -5 $O/sep_$rep.err; exit 1; }
  show $O/sep_$rep.jsonl sep
done
