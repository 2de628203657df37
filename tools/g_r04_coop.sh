set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_coop
timeout -k 10 300 python -u -m pytest tests/test_gpu_insite.py -x -q -k "cooperative or four_arms or dense" > gpurun_out/r04_coop/tests.txt 2>&1 || { tail -40 gpurun_out/r04_coop/tests.txt; exit 1; }
tail -2 gpurun_out/r04_coop/tests.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_refine_general.py tests/test_gpu_reference_segments.py -x -q > gpurun_out/r04_coop/tests2.txt 2>&1 || { tail -40 gpurun_out/r04_coop/tests2.txt; exit 1; }
tail -2 gpurun_out/r04_coop/tests2.txt
timeout -k 10 400 python bench.py --config insite4 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r04_coop/insite4.jsonl 2> gpurun_out/r04_coop/insite4.err || { tail -5 gpurun_out/r04_coop/insite4.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r04_coop/insite4.jsonl').read().strip().splitlines()[-1])
print({k:(round(v['ms_per_step'],2), round(v['kernel_ms'],2), round(v['frac'],4)) for k,v in d['models'].items()})"
