#!/bin/bash
# Same-box A/B of the -J^T F GEMV in the J^T J's tail (PNOL_JTR_TAIL=1, default) against the
# plain stream order (=0): alternating short bench runs, LM iters/s and ms per trip each.
set -u
mkdir -p gpurun_out
for rep in 1 2 3; do
  for t in 1 0; do
    PNOL_JTR_TAIL=$t timeout -k 10 180 python bench.py --no-cpu-baseline --no-hg --no-bfgs --steps 30 --warmup 3 \
        > gpurun_out/ab_tail$t.json 2> gpurun_out/ab_tail$t.err
    rc=$?; [ "$rc" -eq 0 ] || { echo "bench rc=$rc"; tail -5 gpurun_out/ab_tail$t.err; exit $rc; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_tail$t.json')); print('tail=$t', round(d['value'],2), round(d['ms_per_step'],4))"
  done
done
