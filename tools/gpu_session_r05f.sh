#!/bin/bash
# -J^T F folded into the SYRK's diagonal tiles: the LM / J^T F / MPI tests, then same-box library
# A/B on short LM benches (in-tree vs _ab/base = the previous commit), then a kernel trace.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "jtr or lm_ or levmarq or fd_normal or normal or trip or user_program" > gpurun_out/pytest_r05f.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed" gpurun_out/pytest_r05f.log | tail -4; [ "$rc" -eq 0 ] || exit $rc
LIBS=base bash tools/lib_ab.sh
mkdir -p gpurun_out/prof_r05f
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05f -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-hg --no-bfgs > gpurun_out/prof_r05f.json 2> gpurun_out/prof_r05f.err
echo "rocprof rc=$?"
