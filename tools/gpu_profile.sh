#!/bin/bash
# One profiling session for the committed evidence (profiles/rNN_*): fp64 peak microbenchmark,
# the default bench line, rocprofv3 kernel stats of the same bench command, separate PMC passes
# (FETCH_SIZE / WRITE_SIZE) and the 2-rank host-communicator rehearsal of the N > 1 line.
# Every GPU step has its own time limit; the first failure ends the session (no retries).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {   # step NAME LIMIT_S CMD...  (stdout/stderr of CMD go where the caller redirects)
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  echo "$name rc=$rc"
  [ "$rc" -eq 0 ] || exit "$rc"
}
if [ "${MB:-1}" = "1" ]; then
  step fp64_peak 120 ./tools/microbench/fp64_peak > gpurun_out/fp64_peak.json 2> gpurun_out/fp64_peak.err
  cat gpurun_out/fp64_peak.json
fi
if [ "${BENCH:-1}" = "1" ]; then
  step bench 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
  tail -c 1500 gpurun_out/bench.json
fi
if [ "${PROF:-1}" = "1" ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-bfgs > gpurun_out/bench_prof.json 2> gpurun_out/prof.err
fi
if [ "${PMC:-1}" = "1" ]; then
  step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o pmc --output-format csv -- \
      python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-bfgs > gpurun_out/pmc_fetch.log 2>&1
  step pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o pmc --output-format csv -- \
      python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-bfgs > gpurun_out/pmc_write.log 2>&1
fi
if [ "${MFMA:-1}" = "1" ]; then
  step pmc_mfma 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_mfma -o pmc \
      --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-bfgs --no-hg \
      > gpurun_out/pmc_mfma.log 2>&1
fi
if [ "${HOSTCOMM:-1}" = "1" ]; then
  step hostcomm2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29517 bench.py --gpus 2 --host-comm --steps 5 --warmup 2 --no-cpu-baseline --no-bfgs \
      > gpurun_out/bench_hostcomm2.json 2> gpurun_out/bench_hostcomm2.err
  tail -c 600 gpurun_out/bench_hostcomm2.json
fi
exit 0
