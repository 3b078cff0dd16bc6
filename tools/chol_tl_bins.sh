#!/bin/bash
# Per-step timelines of the persistent Cholesky for a list of chol_timeline builds (TLS: binary
# suffixes under tools/microbench/chol_timeline_*), alternating, each summarised by
# chol_tl_summary.py; raw JSON under gpurun_out/tl_<suffix>_<rep>.json.
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for s in ${TLS:-f1 f0}; do
    timeout -k 5 60 ./tools/microbench/chol_timeline_$s 2048 > gpurun_out/tl_${s}_$rep.json || exit 1
    echo "$s $(python3 tools/chol_tl_summary.py < gpurun_out/tl_${s}_$rep.json)"
  done
done
