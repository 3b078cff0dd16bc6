#!/bin/bash
# The fused LM trip with its reduce launch writing the Cholesky's matrix: the LM / trip tests,
# then the three trip forms in alternating same-box runs, then a kernel trace of the default.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "trip or lm_ or relaunch or levmarq_mpi_one_rank or levmarq_mpi_trip or cholesky" > gpurun_out/pytest_r05h.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed" gpurun_out/pytest_r05h.log | tail -4; [ "$rc" -eq 0 ] || exit $rc
REPS=4 bash tools/trip_ab.sh
mkdir -p gpurun_out/prof_r05h
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05h -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-hg --no-bfgs > gpurun_out/prof_r05h.json 2> gpurun_out/prof_r05h.err
echo "rocprof rc=$?"
timeout -k 10 300 python tools/rank_model.py --out gpurun_out/r05_rank_model.json > gpurun_out/r05_rank_model.log 2>&1; echo "rank model rc=$?"; tail -5 gpurun_out/r05_rank_model.log
