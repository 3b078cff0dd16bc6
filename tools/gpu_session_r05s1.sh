#!/bin/bash
# Staged-only look-ahead (tiles ready after the cutoff are still staged into LDS):
# tests, timelines against HEAD's build, bench A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "chol or solve or trip or relaunch or levmarq_mpi_m or lm_fused" > gpurun_out/pytest_r05s1.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed" gpurun_out/pytest_r05s1.log | tail -3; [ "$rc" -eq 0 ] || exit $rc
for v in old new stg old new stg; do
  b=./tools/microbench/chol_timeline; [ "$v" = old ] && b=./tools/microbench/chol_timeline_old
  la=48; [ "$v" = stg ] && la=1
  PNOL_CHOL_LOOKAHEAD=$la timeout -k 10 60 $b 2048 > gpurun_out/r05_tl_$v.json || exit $?
  echo "$v $(python3 tools/chol_tl_summary.py < gpurun_out/r05_tl_$v.json)"
done
LIBS=base bash tools/lib_ab.sh || exit $?
