#!/bin/bash
# -J^T F in the SYRK + the fused trip with its reduce launch into the Cholesky's matrix: the LM /
# J^T F / trip / MPI tests; same-box A/B of the library against the previous commit (_ab/base) and
# of the three trip forms; a kernel trace of the default; the fused-pass prefetch sweep; the
# per-rank step model.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "jtr or lm_ or levmarq or fd_normal or normal or trip or relaunch or cholesky or user_program or prefetch_depth or bfgs_pass" > gpurun_out/pytest_r05i.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed" gpurun_out/pytest_r05i.log | tail -4; [ "$rc" -eq 0 ] || exit $rc
LIBS=base bash tools/lib_ab.sh || exit $?
REPS=3 bash tools/trip_ab.sh || exit $?
mkdir -p gpurun_out/prof_r05i
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05i -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-hg --no-bfgs > gpurun_out/prof_r05i.json 2> gpurun_out/prof_r05i.err
echo "rocprof rc=$?"
timeout -k 10 600 python tools/pass_sweep.py PNOL_PASS_PF=1 PNOL_PASS_PF=2 PNOL_PASS_PF=1 PNOL_PASS_PF=2 || exit $?
timeout -k 10 300 python tools/rank_model.py --out gpurun_out/r05_rank_model.json > gpurun_out/r05_rank_model.log 2>&1
echo "rank model rc=$?"; tail -3 gpurun_out/r05_rank_model.log
