#!/bin/bash
# Streamed solve: its parity tests, the one-XCD solve probe, then bench A/B (PNOL_LM_STREAM).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
step pytest_stream 400 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
    -k "${K:-lm_trip_stream or streamed_trip}" > gpurun_out/pytest_stream.log 2>&1 || { tail -30 gpurun_out/pytest_stream.log; exit 1; }
tail -3 gpurun_out/pytest_stream.log
if [ "${PROBE:-1}" = "1" ]; then bash tools/gpu_probe_solve_xcd.sh > gpurun_out/probe_solve_xcd.log 2>&1; echo "probe rc=$?"; cat gpurun_out/probe_solve_xcd.log; fi
for g in 1 2; do
  PNOL_LM_STREAM=0 step bench_base 200 python bench.py --steps ${STEPS:-40} --warmup 5 --no-cpu-baseline --no-hg --no-bfgs > gpurun_out/bench_base_$g.json
  PNOL_LM_STREAM=1 step bench_stream 200 python bench.py --steps ${STEPS:-40} --warmup 5 --no-cpu-baseline --no-hg --no-bfgs > gpurun_out/bench_stream_$g.json
  tail -c 400 gpurun_out/bench_base_$g.json; echo; tail -c 400 gpurun_out/bench_stream_$g.json; echo
done
exit 0
