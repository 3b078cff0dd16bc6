#!/bin/bash
# Look-ahead cutoff with the staged-only mode: per-step timelines at several cutoffs, then a
# same-box LM bench A/B of the two best.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for la in 1 16 32 40 48 56; do
    PNOL_CHOL_LOOKAHEAD=$la timeout -k 10 60 ./tools/microbench/chol_timeline 2048 > gpurun_out/r05_tl_la$la.json || exit $?
    echo "la=$la $(python3 tools/chol_tl_summary.py < gpurun_out/r05_tl_la$la.json)"
  done
done
VAR=PNOL_CHOL_LOOKAHEAD VALS="1 48" KEY=solve bash tools/env_ab.sh || exit $?
