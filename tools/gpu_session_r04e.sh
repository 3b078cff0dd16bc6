#!/bin/bash
# Streamed solve: trip probe, its parity tests + the bounded-BFGS tests, then bench A/B
# (PNOL_LM_STREAM 0 / 1) with the processes left after each bench listed.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
for sz in "3000 257" "16384 2048"; do
  step probe 120 python tools/stream_trip_probe.py $sz 12 >> gpurun_out/stream_probe.jsonl
done
cat gpurun_out/stream_probe.jsonl
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
    -k "${K:-streamed_trip or lm_trip_stream or bnd or recur}" > gpurun_out/pytest_r04e.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_r04e.log | tail -2; [ "$rc" -eq 0 ] || exit $rc
for g in 1 2; do
  for sv in 0 1; do
    PNOL_LM_STREAM=$sv step bench_s$sv 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-hg ${BFGS:---no-bfgs} > gpurun_out/bench_s${sv}_$g.json
    ps -o pid,ppid,etime,cmd -u "$(id -u)" > gpurun_out/ps_after_bench_s${sv}_$g.txt 2>&1 || true
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['frac'])" gpurun_out/bench_s${sv}_$g.json
  done
done
exit 0
