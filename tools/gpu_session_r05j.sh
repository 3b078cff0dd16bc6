#!/bin/bash
# Knob A/Bs on short LM benches (alternating, same box): the chain wave's issue priority
# (PNOL_CHOL_PRIO) and non-temporal SYRK partial stores (PNOL_SYRK_NTS); the solve timeline with
# and without the priority.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
VAR=PNOL_CHOL_PRIO VALS="0 1" KEY=solve bash tools/env_ab.sh || exit $?
VAR=PNOL_SYRK_NTS VALS="0 1" KEY=syrk_reduce bash tools/env_ab.sh || exit $?
for v in 0 1 0 1; do
  PNOL_CHOL_PRIO=$v timeout -k 10 60 ./tools/microbench/chol_timeline 2048 > gpurun_out/r05_tl_prio$v.json || exit $?
  echo "prio=$v $(python3 tools/chol_tl_summary.py < gpurun_out/r05_tl_prio$v.json)"
done
