#!/bin/bash
# after packing the library exponents into dwords (scalar loads in the gram's G-phase / rollout prologues):
# parity + the C2 kernels and bench modes
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02aa}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for op in gram sindy_fit; do
  timeout -k 10 120 python tools/kbench.py --op $op --layout time --iters 50 > $O/kb_$op.json 2>$O/kb_$op.err || { tail -5 $O/kb_$op.err; exit 1; }
  echo "$op $(cat $O/kb_$op.json | tr -d '\n' | cut -c1-120)"
done
timeout -k 10 120 python tools/kbench.py --op rollout --layout time_bits --iters 50 > $O/kb_rollout.json 2>$O/kb_rollout.err || { tail -5 $O/kb_rollout.err; exit 1; }
echo "rollout $(cat $O/kb_rollout.json | tr -d '\n' | cut -c1-120)"
for m in pipeline fused seq; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --mode $m --steps 50 --isolated > $O/$m.log 2>$O/$m.err || { tail -20 $O/$m.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$m.log'));print('$m ms',round(d['ms_per_step'],5),'frac',round(d['roofline']['frac'],3),'iso',{k:round(x,4) for k,x in d.get('isolated',{}).items()})"
done
for gb in 192 256 320; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --mode fused --gram-blocks $gb --steps 50 > $O/fused_$gb.log 2>$O/fused_$gb.err || { tail -20 $O/fused_$gb.err; exit 1; }
  python -c "import json;d=json.load(open('$O/fused_$gb.log'));print('fused gb $gb ms',round(d['ms_per_step'],5),'frac',round(d['roofline']['frac'],3))"
done
echo ALLOK
