#!/bin/bash
# FD Jacobian with 64 points per wave (PNOL_FD_PW=64) against the default 32: same-box bench A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
VAR=PNOL_FD_PW VALS="0 64" KEY=fd_jacobian bash tools/env_ab.sh || exit $?
