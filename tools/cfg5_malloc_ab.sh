#!/bin/bash
# cfg 5 (BFGS_Bnd, n = 16384) under glibc's default malloc vs huge-page heap (glibc 2.35
# tunable) vs a large top pad: is the per-level "other" time the first touch of fresh pages?
set -u
mkdir -p gpurun_out
for mode in default huge pad; do
  case $mode in
    huge) E="GLIBC_TUNABLES=glibc.malloc.hugetlb=1";;
    pad) E="MALLOC_TOP_PAD_=268435456";;
    *) E="X=1";;
  esac
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-hg --steps 2 --warmup 1 > gpurun_out/m_$mode.json 2> gpurun_out/m_$mode.err
  rc=$?; [ "$rc" -eq 0 ] || { echo "bench rc=$rc"; tail -3 gpurun_out/m_$mode.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/m_$mode.json').readline()); b=d['bfgs_bnd_cfg5_solve']; c=d['bfgs_cfg2_solve']
print('$mode', round(b['seconds'],3), round(b['ms_per_iteration'],4), {k: round(v,4) for k,v in b['phases_ms_per_iteration'].items()}, round(b['other_ms_per_iteration'],4), 'cfg2', round(c['ms_per_iteration'],4))"
done
