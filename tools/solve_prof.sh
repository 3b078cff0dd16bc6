#!/bin/bash
# Cholesky tests, solve timings at n = 2048 (method 5), and per-kernel averages of the solve
# launches from a rocprofv3 kernel-stats pass (prep / persist / backward).
set -u
export TMPDIR=/tmp
bash tools/gpu_quick.sh "cholesky or solve or chol" || exit $?
for g in 1 2 3; do timeout -k 10 120 python tools/solve_bench.py 2048 5 2>&1 | tail -1 || exit 1; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/p -o r --output-format csv -- python tools/solve_bench.py 2048 5 > /dev/null 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
for f in glob.glob("/tmp/p/**/r_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "chol" in r["Name"]:
            print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1000, 1))
PY
