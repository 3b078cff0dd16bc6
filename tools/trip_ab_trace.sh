#!/bin/bash
# Same-box A/B of the LM trip's evaluation kernel from rocprofv3 kernel traces of short benches
# (tools/trip_gaps.py: the evaluation's duration and the idle time around it, medians over the
# trips).  VAR / VALS: an env knob and its settings; LIBS: _ab/<name> builds (csrc/Makefile
# OBJDIR=... LIB=... EXTRA=-D...) compared with the in-tree one (PNOL_AMD_LIB).
#   VAR=PNOL_LM_ZEROCOPY VALS="1 0" tools/eval_ab.sh;  VALS= LIBS="skew" tools/eval_ab.sh
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for v in ${VALS-1 0}; do
    env ${VAR:-PNOL_LM_ZEROCOPY}=$v timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/eab_${v}_$rep -o run --output-format csv -- \
        python3 bench.py --no-cpu-baseline --no-hg --no-bfgs --steps 20 --warmup 3 > gpurun_out/eab_${v}_$rep.log 2>&1 || exit 1
    python3 tools/trip_gaps.py gpurun_out/eab_${v}_$rep/run_kernel_trace.csv "${VAR:-PNOL_LM_ZEROCOPY}=$v"
  done
  for l in ${LIBS-}; do
    PNOL_AMD_LIB=_ab/$l/libpnol_amd.so timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/eab_${l}_$rep -o run --output-format csv -- \
        python3 bench.py --no-cpu-baseline --no-hg --no-bfgs --steps 20 --warmup 3 > gpurun_out/eab_${l}_$rep.log 2>&1 || exit 1
    python3 tools/trip_gaps.py gpurun_out/eab_${l}_$rep/run_kernel_trace.csv "lib=$l"
  done
done
