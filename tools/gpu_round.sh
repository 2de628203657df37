#!/bin/bash
# One GPU call: selected parity tests, then bench lines.  Every GPU step has its own time limit and the first
# failure (test failure, crash, timeout) ends the call.
#   OUT=r03_x TESTS="tests/test_gpu_foo.py" BENCH="--config c5;--config c4 --T 60" bash tools/gpu_round.sh
# TESTS="all" runs the whole -m gpu suite; empty skips tests; KSEL is an optional pytest -k expression;
# XFLAG="" runs past the first failure (default -x); CONT=1 goes on to POST / BENCH after test failures.
# POST is an optional command run (under its own time limit) after the tests.  BENCH is a ';'-separated list
# of bench.py argument strings ("default" = the driver's default line).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-round}
mkdir -p "$O"
if [ -n "$TESTS" ]; then
  sel="$TESTS"; [ "$TESTS" = "all" ] && sel="tests"
  timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest $sel -m gpu ${XFLAG--x} -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider ${KSEL:+-k "$KSEL"} > "$O/tests.log" 2>&1
  rc=$?
  grep -cE "PASSED" "$O/tests.log"; grep -E "^(FAILED|ERROR)" "$O/tests.log" | head -20; tail -2 "$O/tests.log"
  # CONT=1: test failures (rc 1) do not stop the call; crashes, timeouts and collection errors do
  if [ $rc -ne 0 ] && ! { [ "$CONT" = 1 ] && [ $rc -eq 1 ]; }; then tail -40 "$O/tests.log"; exit 1; fi
fi
if [ -n "$POST" ]; then
  timeout -k 10 ${POST_LIMIT:-600} bash -c "$POST" > "$O/post.log" 2>&1 || { echo "post failed"; tail -30 "$O/post.log"; exit 1; }
  tail -${POST_TAIL:-10} "$O/post.log"
fi
i=0
IFS=';' read -ra LINES <<< "$BENCH"
for b in "${LINES[@]}"; do
  [ -z "$b" ] && continue
  [ "$b" = "default" ] && b=""
  i=$((i + 1))
  timeout -k 10 ${BENCH_LIMIT:-400} python bench.py $b > "$O/bench_$i.log" 2> "$O/bench_$i.err" || { echo "bench $i failed: $b"; tail -20 "$O/bench_$i.err"; exit 1; }
  echo "bench $i ($b):"; tail -1 "$O/bench_$i.log" | cut -c1-600
done
echo ALLOK
