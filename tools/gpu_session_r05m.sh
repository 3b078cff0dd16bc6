#!/bin/bash
# Critical-first worker claim order in the persistent Cholesky: the Cholesky / solve / LM trip
# tests, the solve timelines with and without it, then same-box bench A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "chol or solve or trip or relaunch or levmarq or lm_" > gpurun_out/pytest_r05m.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed" gpurun_out/pytest_r05m.log | tail -4; [ "$rc" -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  PNOL_CHOL_CRITFIRST=$v timeout -k 10 60 ./tools/microbench/chol_timeline 2048 > gpurun_out/r05_tl_crit$v.json || exit $?
  echo "crit=$v $(python3 tools/chol_tl_summary.py < gpurun_out/r05_tl_crit$v.json)"
done
VAR=PNOL_CHOL_CRITFIRST VALS="0 1" KEY=solve bash tools/env_ab.sh || exit $?
