#!/bin/bash
# Targeted GPU run: the given pytest selection (-k expression) with per-test timeouts, then
# optionally the bench.  Each GPU step has its own time limit; the script stops at the first
# fault / abort / timeout (no retries).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
K="${1:-}"
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ] || [ "$rc" -eq 5 ]; }
if [ -n "$K" ]; then
  timeout -k 10 ${PYT_LIMIT:-900} python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout ${TEST_LIMIT:-300} \
      --timeout-method thread -k "$K" > gpurun_out/pytest_quick.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_quick.log | tail -40
  ok $rc || exit $rc
fi
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 ${BENCH_LIMIT:-600} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; tail -c 4000 gpurun_out/bench.json; tail -5 gpurun_out/bench.err
  ok $rc || exit $rc
fi
exit 0
