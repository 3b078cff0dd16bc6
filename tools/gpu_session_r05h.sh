#!/bin/bash
# Persistent Cholesky worker count on the current chain (timelines, two rounds).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for w in 255 224 192 160 128; do
    PNOL_CHOL5_WORKERS=$w timeout -k 10 60 ./tools/microbench/chol_timeline 2048 > gpurun_out/r05_tl_w$w.json || exit $?
    echo "w=$w $(python3 tools/chol_tl_summary.py < gpurun_out/r05_tl_w$w.json)"
  done
done
