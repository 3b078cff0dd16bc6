#!/bin/bash
# cfg 5 (BFGS_Bnd, n = 16384) with the host-detail clocks (PNOL_BND_DETAIL=1, stderr)
set -u
mkdir -p gpurun_out
PNOL_BND_DETAIL=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-hg --steps 2 --warmup 1 > gpurun_out/d5.json 2> gpurun_out/d5.err
rc=$?; grep "host detail" gpurun_out/d5.err; [ "$rc" -eq 0 ] || exit $rc
python3 -c "
import json; d=json.loads(open('gpurun_out/d5.json').readline()); b=d['bfgs_bnd_cfg5_solve']
print(round(b['seconds'],3), round(b['ms_per_iteration'],4), {k: round(v,4) for k,v in b['phases_ms_per_iteration'].items()}, round(b['other_ms_per_iteration'],4))"
