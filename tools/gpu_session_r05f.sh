#!/bin/bash
# Round-5 final measurement set on the current default path: the whole GPU suite (one process, the
# driver's -x order), the PMC passes, the default bench line (with the CPU baseline) and a
# rocprofv3 kernel trace of the bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_r05f.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed" gpurun_out/pytest_r05f.log | tail -4; [ "$rc" -eq 0 ] || exit $rc
bash tools/gpu_pmc_r05.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_r05f.json 2> gpurun_out/bench_r05f.err
rc=$?; echo "bench rc=$rc"; head -c 400 gpurun_out/bench_r05f.json; echo; [ "$rc" -eq 0 ] || exit $rc
mkdir -p gpurun_out/prof_r05f
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05f -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_prof_r05f.json 2> gpurun_out/prof_r05f.err
echo "rocprof rc=$?"
