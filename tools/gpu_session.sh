#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel stats.  Each GPU step has its
# own time limit; a step that faults, aborts or times out ends the session (no retries).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }   # 1 = test/assert failures, not a fault

if [ "${MB:-0}" = "1" ]; then
  timeout -k 10 120 ./tools/microbench/fp64_peak > gpurun_out/fp64_peak.json 2>&1
  rc=$?; echo "microbench rc=$rc"; cat gpurun_out/fp64_peak.json; [ "$rc" -eq 0 ] || exit $rc
fi
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
ok $rc || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.json
ok $rc || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/prof.err
  rc=$?; echo "rocprof rc=$rc"
fi
if [ "${SWEEP:-0}" = "1" ]; then
  timeout -k 10 600 python tools/sweep_hg.py > gpurun_out/sweep_hg.log 2>&1
  rc=$?; echo "sweep rc=$rc"; cat gpurun_out/sweep_hg.log; [ "$rc" -eq 0 ] || exit $rc
fi
if [ "${PMC:-0}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o pmc --output-format csv -- \
      python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1
  rc=$?; echo "pmc fetch rc=$rc"; [ "$rc" -eq 0 ] || exit $rc
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o pmc --output-format csv -- \
      python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1
  rc=$?; echo "pmc write rc=$rc"; [ "$rc" -eq 0 ] || exit $rc
fi
if [ "${VALU:-0}" = "1" ]; then
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
      SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_valu -o pmc --output-format csv -- \
      python3 tools/fd_only.py 4 > gpurun_out/pmc_valu.log 2>&1
  rc=$?; echo "pmc valu rc=$rc"; [ "$rc" -eq 0 ] || exit $rc
fi
if [ "${MFMA:-0}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_mfma -o pmc \
      --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_mfma.log 2>&1
  rc=$?; echo "pmc mfma rc=$rc"; [ "$rc" -eq 0 ] || exit $rc
fi
if [ "${HOSTCOMM:-0}" = "1" ]; then   # the N>1 bench path rehearsed on one GPU (gloo + host communicator)
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29517 bench.py --gpus 2 --host-comm --steps 5 --warmup 2 --no-cpu-baseline \
      > gpurun_out/bench_hostcomm2.json 2> gpurun_out/bench_hostcomm2.err
  rc=$?; echo "hostcomm rc=$rc"; tail -c 600 gpurun_out/bench_hostcomm2.json; [ "$rc" -eq 0 ] || exit $rc
fi
exit 0
