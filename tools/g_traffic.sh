#!/bin/bash
# PMC traffic of every bench line's kernels: two rocprofv3 passes (FETCH_SIZE, WRITE_SIZE: one counter group
# per run, MI355X_MICROARCH.md) per config over a short bench.py run, then tools/traffic_summary.py.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-traffic}
mkdir -p $O
# CONFIGS: ';'-separated name:bench-arguments specs
IFS=';' read -ra SPECS <<< "${CONFIGS:-c2:--no-north-star;c4:--config c4 --T 60;c5:--config c5;c3:--config c3;f4:--config f4;insite:--config insite}"
for spec in "${SPECS[@]}"; do
  name=${spec%%:*}; argsx=${spec#*:}
  for C in FETCH_SIZE WRITE_SIZE; do
    d=$O/pmc/$name/$( [ $C = FETCH_SIZE ] && echo fetch || echo write )
    timeout -s KILL ${PMC_LIMIT:-150} rocprofv3 --pmc $C -d $d -o run --output-format csv -- python3 bench.py $argsx --no-cpu-baseline --no-parity --steps 5 --warmup 2 > $O/${name}_$C.log 2>&1 || { echo "pmc $name $C failed"; tail -5 $O/${name}_$C.log; exit 1; }
  done
  echo "pmc $name ok"
done
python3 tools/traffic_summary.py $O/pmc > $O/traffic.json && echo ALLOK
