#!/bin/bash
# cfg 5 (BFGS_Bnd, n = 16384) with glibc's default malloc thresholds vs large mmap / trim
# thresholds (no page-fault churn from 128 KB vectors freed and re-allocated every level).
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for mode in default big; do
    if [ $mode = big ]; then E="MALLOC_MMAP_THRESHOLD_=1073741824 MALLOC_TRIM_THRESHOLD_=4294967296"; else E=""; fi
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-hg --steps 3 --warmup 1 > gpurun_out/m.json 2> gpurun_out/m.err
    rc=$?; [ "$rc" -eq 0 ] || { echo "bench rc=$rc"; tail -3 gpurun_out/m.err; exit $rc; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/m.json').readline()); b=d['bfgs_bnd_cfg5_solve']; c=d['bfgs_cfg2_solve']
print('$mode', round(b['seconds'],3), round(b['ms_per_iteration'],4), {k: round(v,4) for k,v in b['phases_ms_per_iteration'].items()}, round(b['other_ms_per_iteration'],4), 'cfg2', round(c['ms_per_iteration'],4))"
  done
done
