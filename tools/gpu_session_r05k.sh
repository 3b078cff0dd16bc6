#!/bin/bash
# -J^T F back on its GEMV (the SYRK fold measured no net gain): the LM / J^T F / trip tests; five
# alternating same-box rounds of the three trip forms; the chain-priority and NTS-partial knob
# A/Bs with the solve timelines; a kernel trace of the default bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "jtr or lm_ or levmarq or fd_normal or normal or trip or relaunch or cholesky" > gpurun_out/pytest_r05k.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed" gpurun_out/pytest_r05k.log | tail -4; [ "$rc" -eq 0 ] || exit $rc
REPS=5 bash tools/trip_ab.sh || exit $?
bash tools/gpu_session_r05j.sh || exit $?
mkdir -p gpurun_out/prof_r05k
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05k -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-hg --no-bfgs > gpurun_out/prof_r05k.json 2> gpurun_out/prof_r05k.err
echo "rocprof rc=$?"
