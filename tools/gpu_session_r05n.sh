#!/bin/bash
# Worker claim orders of the persistent Cholesky (PNOL_CHOL_ORDER 0 by step, 1 critical tasks a
# step early, 2 by tile column): the Cholesky / solve / LM tests under orders 2 and 1, the solve
# timelines, then same-box bench A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for o in 2 1; do
  PNOL_CHOL_ORDER=$o timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
      -k "chol or solve or trip or relaunch or levmarq_mpi_m or lm_fused" > gpurun_out/pytest_r05n_o$o.log 2>&1
  rc=$?; echo "order $o pytest rc=$rc"; grep -E "FAIL|passed|failed" gpurun_out/pytest_r05n_o$o.log | tail -3; [ "$rc" -eq 0 ] || exit $rc
done
for v in 0 2 1 0 2 1; do
  PNOL_CHOL_ORDER=$v timeout -k 10 60 ./tools/microbench/chol_timeline 2048 > gpurun_out/r05_tl_order$v.json || exit $?
  echo "order=$v $(python3 tools/chol_tl_summary.py < gpurun_out/r05_tl_order$v.json)"
done
VAR=PNOL_CHOL_ORDER VALS="0 2 1" KEY=solve bash tools/env_ab.sh || exit $?
