# GPU recipe (round 5): warm-up length vs the measured step -- every line at the default 5 warmup steps and at a
# warm-up of W2 steps (C5 showed 0.79 ms at 5 and 0.71 at 60: the early steps run before the GPU is at its
# steady state).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_warm
mkdir -p $O
run() {  # name, config, warmup
  timeout -k 10 300 python bench.py --config $2 --no-cpu-baseline --no-parity --warmup $3 > $O/$1.jsonl 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline',{})
print(sys.argv[1], d['warmup'], round(d['ms_per_step'],5), 'kern', r.get('avg_launch_ms'))" $O/$1.jsonl
}
run c2_w5 c2 5 && run c2_w200 c2 200 && run c2_w2000 c2 2000 && run c4_w5 c4 5 && run c4_w200 c4 200 && \
run f4_w5 f4 5 && run f4_w200 f4 200 && run in_w5 insite 5 && run in_w40 insite 40 && run c3_w5 c3 5 && run c3_w20 c3 20
