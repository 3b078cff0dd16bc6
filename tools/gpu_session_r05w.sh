#!/bin/bash
# Fused BFGS pass with 32-row tiles at n >= 12288: the BFGS / pass / bounded-solver tests, then the
# pass sweep at the default setting.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "bfgs or pass or hg or cfg5 or bnd or Bnd" > gpurun_out/pytest_r05w.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed" gpurun_out/pytest_r05w.log | tail -3; [ "$rc" -eq 0 ] || exit $rc
PASS_SIZES=4096,8192,16384 timeout -k 10 300 python tools/pass_sweep.py NONE=0 || exit $?
