#!/bin/bash
# Fused BFGS pass row-tile height at n = 4096 / 8192 / 16384 (PNOL_PASS_ROWS), alternating.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
PASS_SIZES=4096,8192,16384 timeout -k 10 900 python tools/pass_sweep.py PNOL_PASS_ROWS=64 PNOL_PASS_ROWS=32 PNOL_PASS_ROWS=256 PNOL_PASS_ROWS=64 PNOL_PASS_ROWS=32 PNOL_PASS_ROWS=256 || exit $?
