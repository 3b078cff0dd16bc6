#!/bin/bash
# The J^T J reduce inside the SYRK's launch (PNOL_LM_REDUCE=tail; PNOL_SYRK_RED_SC1=1 the
# write-through variant): the trip / LM tests, then same-box trip A/B launch / tail / tail_sc1
# and a kernel trace of the tail form.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "trip or lm_fused or relaunch" > gpurun_out/pytest_r05s.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|passed|failed" gpurun_out/pytest_r05s.log | tail -3; [ "$rc" -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in launch tail tail_sc1; do
    case $v in
      launch) envs="PNOL_LM_REDUCE=launch";;
      tail) envs="PNOL_LM_REDUCE=tail PNOL_SYRK_RED_SC1=0";;
      tail_sc1) envs="PNOL_LM_REDUCE=tail PNOL_SYRK_RED_SC1=1";;
    esac
    env $envs timeout -k 10 180 python bench.py --no-cpu-baseline --no-hg --no-bfgs --steps 40 --warmup 5 \
        > gpurun_out/trip_$v.json 2> gpurun_out/trip_$v.err
    rc=$?; [ "$rc" -eq 0 ] || { echo "bench rc=$rc"; tail -5 gpurun_out/trip_$v.err; exit $rc; }
    python3 -c "import json; d=json.loads(open('gpurun_out/trip_$v.json').readline()); k=d['kernel_ms_per_step_max_over_ranks']; b=d['kernel_ms_per_call_warmup_breakdown']; print('$v', round(d['value'],2), round(d['ms_per_step'],4), 'solve', round(b.get('solve',0),4), 'reduce', round(b.get('syrk_reduce',0),4), 'in-step syrk', round(k['syrk'],4), 'fd', round(k['fd_jacobian'],4))"
  done
done
mkdir -p gpurun_out/prof_r05s
PNOL_LM_REDUCE=tail timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05s -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-hg --no-bfgs > gpurun_out/prof_r05s.json 2> gpurun_out/prof_r05s.err
echo "rocprof rc=$?"
