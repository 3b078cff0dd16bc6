#!/bin/bash
# BFGS parity tests, then the cfg 2 / cfg 5 blocks of the bench twice (per-phase ms per iteration).
set -u
mkdir -p gpurun_out
bash tools/gpu_quick.sh "bfgs or Bnd or bnd" || exit $?
for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-hg --steps 3 --warmup 1 > gpurun_out/m.json 2> gpurun_out/m.err
  rc=$?; [ "$rc" -eq 0 ] || { echo "bench rc=$rc"; tail -3 gpurun_out/m.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/m.json').readline()); b=d['bfgs_bnd_cfg5_solve']; c=d['bfgs_cfg2_solve']
print('cfg5', round(b['seconds'],3), round(b['ms_per_iteration'],4), {k: round(v,4) for k,v in b['phases_ms_per_iteration'].items()}, 'other', round(b['other_ms_per_iteration'],4), b['fopt'], b['iterations'], b['evals'], b['max_abs_err_vs_kkt_point'])
print('cfg2', round(c['ms_per_iteration'],4), c['fopt'], c['evals'])"
done
