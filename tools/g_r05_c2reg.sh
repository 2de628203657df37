# GPU recipe (round 5): the C2 line on this tree vs the round-4 insite_hip.hip (variant library r04c2), alternating,
# three runs each on one box -- is the round-5 C2 number (0.073-0.076 ms) a regression or the box?
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_c2reg${TAG}
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
mkdir -p $O
show() { python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],5), round(d['roofline']['avg_launch_ms'],5))" $1 $2; }
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --no-north-star --steps 96 > $O/head_$rep.jsonl 2>$O/head_$rep.err || { tail -5 $O/head_$rep.err; exit 1; }
  show $O/head_$rep.jsonl head
  INSITE_LIB_OVERRIDE=$A/libinsite_hip_r04c2.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --no-north-star --steps 96 > $O/r04_$rep.jsonl 2>$O/r04_$rep.err || { tail -5 $O/r04_$rep.err; exit 1; }
  show $O/r04_$rep.jsonl r04
done
