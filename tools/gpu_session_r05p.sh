#!/bin/bash
# The chain's look-ahead cutoff (PNOL_CHOL_LOOKAHEAD: give up once wave 0 has c columns final)
# on the current factor: solve timelines per cutoff, then same-box bench A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for v in 0 32 40 48 56 64; do
    PNOL_CHOL_LOOKAHEAD=$v timeout -k 10 60 ./tools/microbench/chol_timeline 2048 > gpurun_out/r05_tl_la$v.json || exit $?
    echo "la=$v $(python3 tools/chol_tl_summary.py < gpurun_out/r05_tl_la$v.json)"
  done
done
VAR=PNOL_CHOL_LOOKAHEAD VALS="64 40 52" KEY=solve bash tools/env_ab.sh || exit $?
