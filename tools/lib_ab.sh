#!/bin/bash
# Same-box A/B of library builds on short LM benches: alternating runs of the in-tree build
# ("default") and the _ab/<name> builds in LIBS; LM iters/s, ms per trip, the warmup solve time
# and the in-step SYRK / FD times (the FD time shows the box's drift between runs).
#   LIBS="mp0" tools/lib_ab.sh
set -u
mkdir -p gpurun_out
for rep in 1 2 3; do
  for v in default ${LIBS:-mp0}; do
    if [ "$v" = "default" ]; then lib=""; else lib=_ab/$v/libpnol_amd.so; fi
    PNOL_AMD_LIB=$lib timeout -k 10 180 python bench.py --no-cpu-baseline --no-hg --no-bfgs --steps 30 --warmup 3 \
        > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err
    rc=$?; [ "$rc" -eq 0 ] || { echo "bench rc=$rc"; tail -5 gpurun_out/ab_$v.err; exit $rc; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_$v.json').readline()); k=d['kernel_ms_per_step_max_over_ranks']; print('$v', round(d['value'],2), round(d['ms_per_step'],4), 'solve', round(d['kernel_ms_per_call_warmup_breakdown'].get('solve',0),4), 'in-step syrk', round(k['syrk'],4), 'fd', round(k['fd_jacobian'],4))"
  done
done
