#!/bin/bash
# Same-box A/B of the LM trip forms on short LM benches, alternating: the fused trip with its
# reduce launch into the Cholesky's matrix (default), the two calls (PNOL_LM_TRIP=0), the fused
# trip with the reduce in the persistent launch's tasks (PNOL_LM_REDUCE=tasks).  REPS rounds.
set -u
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-3}); do
  for v in launch two tasks; do
    case $v in
      launch) envs="PNOL_LM_TRIP=1 PNOL_LM_REDUCE=launch";;
      two) envs="PNOL_LM_TRIP=0";;
      tasks) envs="PNOL_LM_TRIP=1 PNOL_LM_REDUCE=tasks";;
    esac
    env $envs timeout -k 10 180 python bench.py --no-cpu-baseline --no-hg --no-bfgs --steps 40 --warmup 5 \
        > gpurun_out/trip_$v.json 2> gpurun_out/trip_$v.err
    rc=$?; [ "$rc" -eq 0 ] || { echo "bench rc=$rc"; tail -5 gpurun_out/trip_$v.err; exit $rc; }
    python3 -c "import json; d=json.loads(open('gpurun_out/trip_$v.json').readline()); k=d['kernel_ms_per_step_max_over_ranks']; b=d['kernel_ms_per_call_warmup_breakdown']; print('$v', round(d['value'],2), round(d['ms_per_step'],4), 'solve', round(b.get('solve',0),4), 'reduce', round(b.get('syrk_reduce',0),4), 'in-step syrk', round(k['syrk'],4), 'fd', round(k['fd_jacobian'],4))"
  done
done
