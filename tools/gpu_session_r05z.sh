#!/bin/bash
# SYRK tile order with the diagonal tiles last (PNOL_SYRK_DLAST=1): trip tests, same-box bench
# A/B, and FETCH_SIZE passes of both orders.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "trip_bitwise or lm_fused" > gpurun_out/pytest_r05z.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed" gpurun_out/pytest_r05z.log | tail -3; [ "$rc" -eq 0 ] || exit $rc
VAR=PNOL_SYRK_DLAST VALS="0 1" KEY=syrk bash tools/env_ab.sh || exit $?
for v in 0 1; do
  PNOL_SYRK_DLAST=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d /tmp/pf$v -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-bfgs --no-hg > gpurun_out/pf$v.log 2>&1 || exit $?
  python3 - <<PY
import csv, glob
v=[float(r['Counter_Value']) for f in glob.glob('/tmp/pf$v/**/*counter_collection.csv', recursive=True) for r in csv.DictReader(open(f)) if 'k_syrk_red' in r.get('Kernel_Name','')]
print('dlast=$v syrk_red FETCH (x2) MB per launch', round(2*sum(v)/len(v)/1e3, 1) if v else None, len(v))
PY
done
