#!/bin/bash
# Micro-panel factor with the deferred rank-1 update three pivots behind (PNOL_MP_DEF=3, in-tree
# build) against two (_ab/base, *_old): Cholesky tests, the factor probe, timelines, bench A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "chol or solve or trip or relaunch or lm_fused or levmarq" > gpurun_out/pytest_r05s4.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed" gpurun_out/pytest_r05s4.log | tail -3; [ "$rc" -eq 0 ] || exit $rc
for v in old new old new; do
  timeout -k 10 60 ./tools/microbench/diag_factor_probe_$v > gpurun_out/r05_diagprobe_$v.json || exit $?
  echo "probe $v $(head -c 600 gpurun_out/r05_diagprobe_$v.json)"
done
for v in old new old new; do
  b=./tools/microbench/chol_timeline; [ "$v" = old ] && b=./tools/microbench/chol_timeline_old
  timeout -k 10 60 $b 2048 > gpurun_out/r05_tl_$v.json || exit $?
  echo "$v $(python3 tools/chol_tl_summary.py < gpurun_out/r05_tl_$v.json)"
done
LIBS=base bash tools/lib_ab.sh || exit $?
