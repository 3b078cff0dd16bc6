#!/bin/bash
# The chain wave's idle lanes forming V_1..V_3 (+ W block rows stored as they become final):
# the Cholesky / LM tests, the diagonal factor probe and the solve timeline (old vs new), then
# same-box library A/B on short LM benches (in-tree vs _ab/base).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "cholesky or solve or lm_trip or chol or relaunch or levmarq_mpi_one_rank or matrix_inverse" > gpurun_out/pytest_r05d.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed" gpurun_out/pytest_r05d.log | tail -4; [ "$rc" -eq 0 ] || exit $rc
for v in old new old new; do
  timeout -k 10 60 ./tools/microbench/diag_factor_probe_$v > gpurun_out/r05_diagprobe_$v.json; rc=$?; [ "$rc" -eq 0 ] || exit $rc
  echo "diag $v $(cat gpurun_out/r05_diagprobe_$v.json | head -c 600)"
done
for v in old new old new; do
  timeout -k 10 60 ./tools/microbench/chol_timeline_$v 2048 > gpurun_out/r05_tl_$v.json; rc=$?; [ "$rc" -eq 0 ] || exit $rc
  python3 tools/chol_tl_summary.py < gpurun_out/r05_tl_$v.json 2>&1 | tail -3
done
LIBS=base bash tools/lib_ab.sh
