#!/bin/bash
# One parameterised GPU session (replaces the per-round gpu_session_rNN*.sh one-offs).  Every GPU
# step has its own time limit; a step that faults, aborts or times out ends the session (no
# retries).  Outputs go to gpurun_out/<TAG>_*.
#
#   TAG=r06a                        output prefix (default: s)
#   TESTS="-k 'trip or chol'"       pytest selection of the -m gpu suite; TESTS=all the whole
#                                   suite; TESTS=none (default) skips the tests
#   SMOKE=1                         __graft_entry__.smoke()
#   BENCH=1 (default)               the default bench line (N = 1)
#   BENCH_ARGS="--no-bfgs ..."      extra bench arguments
#   PROFILE=1                       rocprofv3 --kernel-trace --stats of the bench command
#   PMC=1 / MFMA=1 / VALU=1         FETCH_SIZE + WRITE_SIZE passes / MFMA busy / FD VALU passes
#   AB_VAR=PNOL_X AB_VALS="0 1"     same-box A/B of an env knob (tools/env_ab.sh, KEY= its timer)
#   HOSTCOMM=1                      the N > 1 bench line rehearsed on one GPU (host communicator)
#   MB=1                            the fp64 peak microbenchmark
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-s}
stop() { echo "$1 rc=$2"; exit "$2"; }

if [ "${MB:-0}" = "1" ]; then
  timeout -k 10 120 ./tools/microbench/fp64_peak > gpurun_out/${T}_fp64_peak.json 2>&1
  rc=$?; echo "microbench rc=$rc"; cat gpurun_out/${T}_fp64_peak.json; [ "$rc" -eq 0 ] || stop microbench $rc
fi
TESTS=${TESTS:-none}
if [ "$TESTS" != "none" ]; then
  sel=""; [ "$TESTS" = "all" ] || sel="$TESTS"
  eval timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
      --timeout-method thread $sel > gpurun_out/${T}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed" gpurun_out/${T}_pytest.log | tail -20
  [ "$rc" -eq 0 ] || stop pytest $rc
fi
if [ "${SMOKE:-0}" = "1" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${T}_smoke.log; [ "$rc" -eq 0 ] || stop smoke $rc
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
  rc=$?; echo "bench rc=$rc"; head -c 600 gpurun_out/${T}_bench.json; echo; [ "$rc" -eq 0 ] || stop bench $rc
fi
if [ "${PROFILE:-0}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- \
      python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/${T}_bench_prof.json \
      2> gpurun_out/${T}_prof.err
  rc=$?; echo "rocprof rc=$rc"; [ "$rc" -eq 0 ] || stop rocprof $rc
  python3 tools/prof_summary.py gpurun_out/${T}_prof > gpurun_out/${T}_prof_summary.txt 2>&1 && \
      head -40 gpurun_out/${T}_prof_summary.txt
fi
pmc() {   # name, counters..., one pass per call
  local name=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" -d gpurun_out/${T}_pmc_$name -o pmc --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_pmc_$name.log 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; [ "$rc" -eq 0 ] || stop "pmc $name" $rc
}
if [ "${PMC:-0}" = "1" ]; then pmc fetch FETCH_SIZE; pmc write WRITE_SIZE; fi
if [ "${MFMA:-0}" = "1" ]; then pmc mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE; fi
if [ "${VALU:-0}" = "1" ]; then
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
      SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/${T}_pmc_valu -o pmc --output-format csv -- \
      python3 tools/fd_only.py 4 > gpurun_out/${T}_pmc_valu.log 2>&1
  rc=$?; echo "pmc valu rc=$rc"; [ "$rc" -eq 0 ] || stop "pmc valu" $rc
fi
if [ -n "${AB_VAR:-}" ]; then
  VAR=$AB_VAR VALS="${AB_VALS:-0 1}" KEY=${KEY:-syrk} bash tools/env_ab.sh 2>&1 | tee gpurun_out/${T}_ab.txt
  rc=${PIPESTATUS[0]}; [ "$rc" -eq 0 ] || stop ab $rc
fi
if [ "${HOSTCOMM:-0}" = "1" ]; then
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29517 bench.py --gpus 2 --host-comm --steps 5 --warmup 2 --no-cpu-baseline \
      > gpurun_out/${T}_bench_hostcomm2.json 2> gpurun_out/${T}_bench_hostcomm2.err
  rc=$?; echo "hostcomm rc=$rc"; tail -c 600 gpurun_out/${T}_bench_hostcomm2.json; [ "$rc" -eq 0 ] || stop hostcomm $rc
fi
exit 0
