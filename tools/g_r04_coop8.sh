set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_coop8
mkdir -p $O
INSITE_REFINE_COOP8=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_insite.py tests/test_gpu_refine_general.py tests/test_gpu_reference_segments.py -x -q --timeout 300 > $O/tests_coop8.txt 2>&1; echo "coop8 tests rc $?"; tail -3 $O/tests_coop8.txt
for rep in 1 2; do
for var in 1 0; do
  INSITE_REFINE_COOP8=$var timeout -k 10 400 python bench.py --config insite4 --no-cpu-baseline --steps 3 --warmup 1 > $O/insite4_coop8_${var}_$rep.jsonl 2>/dev/null || exit 1
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('coop8', sys.argv[2], {k:(round(v['ms_per_step'],2), round(v['kernel_ms'],2), v['kernel'], round(v['mean_evaluations_per_refined_row'],4)) for k,v in d['models'].items() if k=='sparse'})" $O/insite4_coop8_${var}_$rep.jsonl $var
done
done
