#!/bin/bash
# Same-box A/B: the default bench (FD / SYRK timer events in the timed region) vs --no-timers.
set -u
mkdir -p gpurun_out
for rep in 1 2 3; do
  for t in "" "--no-timers"; do
    timeout -k 10 180 python bench.py --no-cpu-baseline --no-hg --no-bfgs --steps 30 --warmup 3 $t > gpurun_out/ab_t.json 2> gpurun_out/ab_t.err
    rc=$?; [ "$rc" -eq 0 ] || { echo "bench rc=$rc"; tail -5 gpurun_out/ab_t.err; exit $rc; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_t.json').readline()); print('timers ${t:-on}', round(d['value'],2), round(d['ms_per_step'],4))"
  done
done
