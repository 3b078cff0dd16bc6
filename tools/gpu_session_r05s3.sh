#!/bin/bash
# The trip's SYRK sub-chunk count (PNOL_SYRK_SUB) with the in-launch reduce: same-box LM A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
VAR=PNOL_SYRK_SUB VALS="2 1 3 4" KEY=syrk bash tools/env_ab.sh || exit $?
