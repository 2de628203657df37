#!/bin/bash
# GPU recipe (round 6): tile-major bit arms -- parity tests of every bit-arm rollout on both layouts, then the A/B of
# the north-star step (--ns-arms), the C2 line and C4 (--arm-format) on time-major vs tile-major bits, and the PMC
# traffic of the north-star step on each layout (FETCH_SIZE / WRITE_SIZE in separate passes).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06_h${TAG}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_tile_bits.py \
  tests/test_gpu_deferred.py tests/test_gpu_refit_rollout.py > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
show() { python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline',{})
print(sys.argv[2], round(d['ms_per_step'],5), round(r.get('avg_launch_ms',0),5), round(r.get('frac',0),4))" $1 $2; }
for rep in 1 2; do
  for f in bits tiles; do
    timeout -k 10 240 python bench.py --config ns --ns-arms $f --no-cpu-baseline --no-parity --steps 20 --warmup 5 > $O/ns_${f}_$rep.jsonl 2> $O/ns_${f}_$rep.err || { tail -5 $O/ns_${f}_$rep.err; exit 1; }
    show $O/ns_${f}_$rep.jsonl ns_${f}_$rep
    timeout -k 10 200 python bench.py --arm-format $f --no-cpu-baseline --no-parity --no-north-star --no-c3-block --steps 100 --warmup 20 > $O/c2_${f}_$rep.jsonl 2> $O/c2_${f}_$rep.err || { tail -5 $O/c2_${f}_$rep.err; exit 1; }
    show $O/c2_${f}_$rep.jsonl c2_${f}_$rep
  done
done
for f in bits tiles; do
  timeout -k 10 240 python bench.py --config c4 --T 60 --arm-format $f --no-cpu-baseline --no-parity --steps 20 --warmup 5 > $O/c4_${f}.jsonl 2> $O/c4_${f}.err || { tail -5 $O/c4_${f}.err; exit 1; }
  show $O/c4_${f}.jsonl c4_${f}
done
# parity line of the north-star step on tile bits (oracle check at the full size)
timeout -k 10 300 python bench.py --config ns --ns-arms tiles --no-cpu-baseline --steps 10 --warmup 3 > $O/ns_tiles_parity.jsonl 2> $O/ns_tiles_parity.err || { tail -5 $O/ns_tiles_parity.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/ns_tiles_parity.jsonl').read().strip().splitlines()[-1]); print('nsparity', d.get('parity'))"
for f in bits tiles; do
  for C in FETCH_SIZE WRITE_SIZE; do
    d=$O/pmc/ns_$f/$( [ $C = FETCH_SIZE ] && echo fetch || echo write )
    timeout -s KILL 150 rocprofv3 --pmc $C -d $d -o run --output-format csv -- python3 bench.py --config ns --ns-arms $f --no-cpu-baseline --no-parity --steps 5 --warmup 2 > $O/pmc_ns_${f}_$C.log 2>&1 || { echo "pmc ns $f $C failed"; tail -5 $O/pmc_ns_${f}_$C.log; exit 1; }
  done
done
python3 tools/traffic_summary.py $O/pmc > $O/traffic.json && echo HDONE
