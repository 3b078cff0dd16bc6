# The whole GPU test suite (one process, per-test limits), then smoke(); stops at the first failure.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_full.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAIL|ERROR|passed|failed" gpurun_out/pytest_full.log | tail -20; [ "$rc" -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; exit $rc
