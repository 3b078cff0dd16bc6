#!/bin/bash
# The diagonal factor alone with the deferral at 3 pivots (diag_factor_probe_new) vs 2 (_old).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in old new old new; do
  timeout -k 10 60 ./tools/microbench/diag_factor_probe_$v > gpurun_out/r05_diagprobe_$v.json || exit $?
  echo "probe $v $(head -c 900 gpurun_out/r05_diagprobe_$v.json)"
done
