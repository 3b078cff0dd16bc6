#!/bin/bash
# Recur gradient: frozen coordinates evaluated with their last real step (the unwinding
# recursion's same-point calls then find every freed coordinate cached).  BFGS / bounded tests,
# then cfg-5 solves alternating with the previous build (_ab/base).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "bfgs or Bnd or bnd or recur or Recur" > gpurun_out/pytest_r05y.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed" gpurun_out/pytest_r05y.log | tail -3; [ "$rc" -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in default base; do
    if [ "$v" = default ]; then lib=""; else lib=_ab/base/libpnol_amd.so; fi
    PNOL_AMD_LIB=$lib timeout -k 10 120 python tools/cfg5_only.py > gpurun_out/c5_$v.json 2> gpurun_out/c5_$v.err
    rc=$?; [ "$rc" -eq 0 ] || { echo "cfg5 rc=$rc"; tail -3 gpurun_out/c5_$v.err; exit $rc; }
    python3 -c "
import json; b=json.loads(open('gpurun_out/c5_$v.json').read().strip().splitlines()[-1])
print('$v', round(b['seconds'],3), round(b['ms_per_iteration'],4), {k: round(v,4) for k,v in b['phases_ms_per_iteration'].items()}, b['iterations'], b['evals'], b['fopt'], round(b['iteration_over_kernel_sum'],2))"
  done
done
