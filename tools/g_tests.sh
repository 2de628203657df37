set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu ${PYTEST_EXTRA:-} > gpurun_out/t_all.log 2>&1 || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/t_all.log | head -40; tail -5 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
