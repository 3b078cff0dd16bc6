#!/bin/bash
# Round 5: the cfg-5 tests (tightened KKT bound, n = 2048 oracle), then the fused trip vs the two
# calls (PNOL_LM_TRIP 1 / 0) in 5 alternating same-box pairs, then a kernel trace of the default.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "cfg5 or unphased" > gpurun_out/pytest_r05b.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|passed|failed" gpurun_out/pytest_r05b.log | tail -8; [ "$rc" -eq 0 ] || exit $rc
for g in 1 2 3 4 5; do
  for tv in 1 0; do
    PNOL_LM_TRIP=$tv timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-hg --no-bfgs > gpurun_out/ab_trip${tv}_$g.json 2> gpurun_out/ab_trip${tv}_$g.err
    rc=$?; [ "$rc" -eq 0 ] || { echo "bench rc=$rc"; tail -5 gpurun_out/ab_trip${tv}_$g.err; exit $rc; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value'],1), round(d['ms_per_step'],3), round(d['roofline']['frac'],3))" gpurun_out/ab_trip${tv}_$g.json
  done
done
mkdir -p gpurun_out/prof_r05b
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05b -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-hg --no-bfgs > gpurun_out/prof_r05b.json 2> gpurun_out/prof_r05b.err
echo "rocprof rc=$?"
find gpurun_out/prof_r05b -name "*stats*" | head
exit 0
