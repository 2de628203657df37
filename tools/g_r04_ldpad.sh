set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_ldpad
mkdir -p $O
for rep in 1 2; do
for pad in 0 32 64 128 256 512 1024; do
  INSITE_TM_LDPAD=$pad timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --steps 100 --warmup 10 > $O/pad${pad}_$rep.jsonl 2>$O/pad${pad}_$rep.err || { tail -5 $O/pad${pad}_$rep.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('pad', sys.argv[2], round(d['ms_per_step'],5), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_ms'],5), d.get('parity',{}).get('support_equal'))" $O/pad${pad}_$rep.jsonl $pad
done
done
