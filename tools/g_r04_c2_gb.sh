set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_c2gb
for rep in 1 2; do
for G in 0 256 304 320 336 352 384 416 448; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --gram-blocks $G --steps 100 --warmup 10 > gpurun_out/r04_c2gb/gb${G}_$rep.jsonl 2>/dev/null || exit 1
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('rep', sys.argv[3], 'gram_blocks', sys.argv[2], round(d['ms_per_step'],5), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_ms'],5))" gpurun_out/r04_c2gb/gb${G}_$rep.jsonl $G $rep
done
done
