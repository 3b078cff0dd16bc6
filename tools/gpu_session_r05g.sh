#!/bin/bash
# The round's committed bench line and its rocprofv3 kernel trace, after the PMC files of the
# same build were committed under profiles/ (the bench reads traffic / MFMA busy from them).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_r05g.json 2> gpurun_out/bench_r05g.err
rc=$?; echo "bench rc=$rc"; head -c 400 gpurun_out/bench_r05g.json; echo; [ "$rc" -eq 0 ] || exit $rc
mkdir -p gpurun_out/prof_r05g
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05g -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_prof_r05g.json 2> gpurun_out/prof_r05g.err
echo "rocprof rc=$?"
