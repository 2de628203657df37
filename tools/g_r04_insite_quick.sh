set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_iq
timeout -k 10 400 python -u -m pytest tests/test_gpu_insite.py tests/test_gpu_refine_general.py tests/test_gpu_reference.py -x -q > gpurun_out/r04_iq/tests.txt 2>&1 || { tail -30 gpurun_out/r04_iq/tests.txt; exit 1; }
tail -2 gpurun_out/r04_iq/tests.txt
for e in INSITE_REFINE_DYN=0 INSITE_REFINE_DYN=1; do
  timeout -k 10 200 env $e python bench.py --config insite --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/r04_iq/$e.jsonl 2>/dev/null || exit 1
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],3), round(d['roofline']['avg_launch_ms'],3))" gpurun_out/r04_iq/$e.jsonl $e
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r04_iq/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config insite --no-cpu-baseline --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/r04_iq/prof.log 2>&1 && echo PROF ok
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --config insite4 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r04_iq/insite4.jsonl 2> gpurun_out/r04_iq/insite4.err || { tail -5 gpurun_out/r04_iq/insite4.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04_iq/insite4.jsonl').read().strip().splitlines()[-1])
print({k:(round(v['ms_per_step'],2), round(v['kernel_ms'],2)) for k,v in d['models'].items()})"
