#!/bin/bash
# The backward solve with two block rows per workgroup: Cholesky / solve / LM tests, solve
# timelines and bench A/B against one block row per workgroup (PNOL_BWD_PAIRS=0).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "chol or solve or trip or relaunch or lm_fused" > gpurun_out/pytest_r05u.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed" gpurun_out/pytest_r05u.log | tail -3; [ "$rc" -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  PNOL_BWD_PAIRS=$v timeout -k 10 60 ./tools/microbench/chol_timeline 2048 > gpurun_out/r05_tl_bwd$v.json || exit $?
  echo "pairs=$v $(python3 tools/chol_tl_summary.py < gpurun_out/r05_tl_bwd$v.json)"
done
VAR=PNOL_BWD_PAIRS VALS="0 1" KEY=solve bash tools/env_ab.sh || exit $?
