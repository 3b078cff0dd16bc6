#!/bin/bash
# Committed-evidence session (profiles/rNN_*): the default bench line, rocprofv3 kernel stats of
# a bench command (the trace itself is dropped: only the stats travel back), separate PMC passes
# (FETCH_SIZE, WRITE_SIZE; MFMA busy) summarised on the box, raw counter files deleted so the
# merged gpurun_out/ stays small.  Each GPU step has its own limit; the first failure ends it.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
exec 3>&1   # the session's stdout: step status lines stay out of the redirected outputs
step() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@"
  local rc=$?
  echo "$name rc=$rc" >&3
  [ "$rc" -eq 0 ] || exit "$rc"
}
if [ "${BENCH:-1}" = "1" ]; then
  step bench 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
  head -c 1200 gpurun_out/bench.json; echo
  tail -c 300000 gpurun_out/bench.err > gpurun_out/bench.err.tail && mv gpurun_out/bench.err.tail gpurun_out/bench.err
fi
if [ "${PROF:-1}" = "1" ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run --output-format csv -- \
      python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-bfgs > gpurun_out/bench_prof.json 2> /tmp/prof.err
  mkdir -p gpurun_out/prof
  find /tmp/prof -name "run_kernel_stats.csv" -exec cp {} gpurun_out/prof/ \;
  head -c 600 gpurun_out/bench_prof.json; echo
fi
if [ "${PMC:-1}" = "1" ]; then
  step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d /tmp/pmc_fetch -o pmc --output-format csv -- \
      python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-bfgs > /tmp/pmc_fetch.log 2>&1
  step pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d /tmp/pmc_write -o pmc --output-format csv -- \
      python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-bfgs > /tmp/pmc_write.log 2>&1
  # the sliced SYRK an N > 1 rank runs (k_syrk_tile<4, 64>), in one process over all 8 m-slices
  step pmc_fetch_sliced 300 rocprofv3 --pmc FETCH_SIZE -d /tmp/pmc_fetch -o probe --output-format csv -- \
      python tools/syrk_sliced_probe.py 3 > /tmp/pmc_fetch_sliced.log 2>&1
  step pmc_write_sliced 300 rocprofv3 --pmc WRITE_SIZE -d /tmp/pmc_write -o probe --output-format csv -- \
      python tools/syrk_sliced_probe.py 3 > /tmp/pmc_write_sliced.log 2>&1
  python3 tools/pmc_traffic.py /tmp/pmc_fetch /tmp/pmc_write gpurun_out/pmc_traffic.json
fi
if [ "${MFMA:-1}" = "1" ]; then
  step pmc_mfma 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d /tmp/pmc_mfma -o pmc \
      --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-bfgs --no-hg \
      > /tmp/pmc_mfma.log 2>&1
  python3 tools/pmc_valu.py /tmp/pmc_mfma gpurun_out/pmc_syrk_mfma.json k_syrk_tile
fi
exit 0
