#!/bin/bash
# C2 discovery parity tests + bench (pipeline, seq) + A/B variants + kernel stats
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-c2f}
A=$GRAFT_REPO_ROOT/ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd/lib/ablate
mkdir -p $O
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_insite.py tests/test_gpu_plugin.py} -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/c2.log 2>$O/c2.err || { tail -20 $O/c2.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-north-star --mode seq > $O/c2_seq.log 2>$O/c2_seq.err || { tail -20 $O/c2_seq.err; exit 1; }
for v in ${VARIANTS}; do INSITE_LIB_OVERRIDE=$A/libinsite_hip_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-north-star > $O/c2_$v.log 2>$O/c2_$v.err || { tail -20 $O/c2_$v.err; exit 1; }; INSITE_LIB_OVERRIDE=$A/libinsite_hip_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-north-star --mode seq > $O/c2_seq_$v.log 2>$O/c2_seq_$v.err || { tail -20 $O/c2_seq_$v.err; exit 1; }; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-north-star > $O/c2_prof.log 2>&1 || { tail -20 $O/c2_prof.log; exit 1; }
for f in $O/c2*.log; do python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; q=d['discovery']
print(sys.argv[1], d['config']['mode'], round(d['ms_per_step']*1e3,1), 'us/step roll', round(r['avg_launch_ms']*1e3,1), round(r['frac'],3), 'disc', round(q['avg_ms']*1e3,1), round(q['frac'],3))" $f 2>/dev/null; done
echo ALLOK
