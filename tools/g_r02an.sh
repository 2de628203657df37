#!/bin/bash
# pipeline batch size K / rollout streams RS sweep, same box, 2 rounds
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r02an}
mkdir -p $O
for r in 1 2; do
for kr in "4 2" "2 2" "8 2" "4 3" "8 3" "16 2"; do
  set -- $kr
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-north-star --no-fused --steps 96 --pipe-k $1 --pipe-rs $2 > $O/k$1_rs$2_$r.log 2>$O/err || { tail -5 $O/err; exit 1; }
  python -c "import json;d=json.load(open('$O/k$1_rs$2_$r.log'));print('K $1 RS $2 r $r ms',round(d['ms_per_step'],5),d['config']['discovered_support'][1])"
done
done
echo ALLOK
