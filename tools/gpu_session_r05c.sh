#!/bin/bash
# LM tests after the trip-form default change, then the default bench line.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "relaunch or lm_ or levmarq or cholesky or trip" > gpurun_out/pytest_r05c.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed" gpurun_out/pytest_r05c.log | tail -4; [ "$rc" -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-hg --no-bfgs > gpurun_out/bench_r05c.json 2> gpurun_out/bench_r05c.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench_r05c.json
