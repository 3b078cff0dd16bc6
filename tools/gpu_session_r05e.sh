#!/bin/bash
# Fused BFGS pass prefetch depth: bitwise test, then alternating sweeps PF 1 / 2.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
    -k "prefetch_depth or bfgs_pass or fused_pass" > gpurun_out/pytest_r05e.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed" gpurun_out/pytest_r05e.log | tail -4; [ "$rc" -eq 0 ] || exit $rc
timeout -k 10 600 python tools/pass_sweep.py PNOL_PASS_PF=1 PNOL_PASS_PF=2 PNOL_PASS_PF=1 PNOL_PASS_PF=2 PNOL_PASS_PF=1 PNOL_PASS_PF=2
