#!/bin/bash
# The LM trip with the Cholesky gated into the J^T J's tail: its parity tests and the LM tests,
# then bench A/B over (trip + tail gate) / (trip, stream order) / (two calls), alternating, and
# a kernel trace of the default trip.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
    -k "${K:-lm_trip or lm_ or levmarq or cholesky}" > gpurun_out/pytest_r04g.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_r04g.log | tail -2; [ "$rc" -eq 0 ] || exit $rc
for g in 1 2; do
  for cfg in "1 1" "1 0" "0 1"; do
    set -- $cfg
    PNOL_LM_TRIP=$1 PNOL_LM_TAIL=$2 timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-hg --no-bfgs > gpurun_out/bench_g$1$2_$g.json 2> gpurun_out/bench_g$1$2_$g.err
    rc=$?; [ "$rc" -eq 0 ] || { echo "bench rc=$rc"; exit $rc; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), round(d['ms_per_step'],3), round(d['roofline']['frac'],3))" gpurun_out/bench_g$1$2_$g.json
  done
done
mkdir -p gpurun_out/prof_tail
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tail -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-hg --no-bfgs > gpurun_out/prof_tail.json 2> gpurun_out/prof_tail.err
echo "rocprof rc=$?"
exit 0
