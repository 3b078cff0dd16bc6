#!/bin/bash
# Cholesky A/B: the microbenchmarks named in DIAGS (binaries under tools/microbench, none by
# default), the Cholesky / LM GPU tests on the default build, then alternating solve timings at n = 2048
# (method 5) of the default library and the _ab/<name> builds listed in LIBS.  Each GPU step has
# its own limit; the first failure ends the session.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@"; local rc=$?; echo "$name rc=$rc"; [ "$rc" -eq 0 ] || exit "$rc"; }
for b in ${DIAGS:-}; do step "$b" 60 ./tools/microbench/$b; done
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
      -k "${K:-cholesky or solve or lm_}" > gpurun_out/pytest_chol.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_chol.log; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ] || exit $rc
fi
for g in 1 2 3; do
  step solve_default 120 python tools/solve_bench.py 2048 5
  for v in ${LIBS:-}; do
    PNOL_AMD_LIB=_ab/$v/libpnol_amd.so step "solve_$v" 120 python tools/solve_bench.py 2048 5
  done
done
exit 0
