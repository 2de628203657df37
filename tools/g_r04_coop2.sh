set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_coop2
timeout -k 10 120 python tools/coop_diag.py | grep differing && DIAG_N=2000 DIAG_JOINT=1 timeout -k 10 120 python tools/coop_diag.py | grep differing || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_insite.py tests/test_gpu_refine_general.py tests/test_gpu_reference_segments.py -x -q > gpurun_out/r04_coop2/tests.txt 2>&1 || { tail -40 gpurun_out/r04_coop2/tests.txt; exit 1; }
tail -2 gpurun_out/r04_coop2/tests.txt
timeout -k 10 200 python bench.py --config insite --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/r04_coop2/insite.jsonl 2>/dev/null || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/r04_coop2/insite.jsonl').read().strip().splitlines()[-1]); print('insite', round(d['ms_per_step'],3), round(d['roofline']['avg_launch_ms'],3))"
timeout -k 10 400 python bench.py --config insite4 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r04_coop2/insite4.jsonl 2> gpurun_out/r04_coop2/insite4.err || { tail -5 gpurun_out/r04_coop2/insite4.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04_coop2/insite4.jsonl').read().strip().splitlines()[-1])
print({k:(round(v['ms_per_step'],2), round(v['kernel_ms'],2), round(v['frac'],4)) for k,v in d['models'].items()})"
